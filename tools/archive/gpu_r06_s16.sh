#!/bin/bash
# Round 6 step 16: the dot-key forward cell through the clamped builtin (SED_DOT_BUILTIN=1: the compiler schedules the
# dots and inserts their wait states, no fences and no fence s_nops): the route and parity tests on that build
# (SED_LIBRARY), its SQ pass, and c4 A/B against the default
set -e
O=$PWD/gpurun_out/${1:-r06s16}
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/tools/ab_libs/libsed_db1.so
SED_LIBRARY=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or parity" > $O/tests_db1.log 2>&1
tail -2 $O/tests_db1.log
SED_LIBRARY=$V timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -d $O/sq_db1 -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_db1.json 2> $O/sq_db1.log
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s16}/c4 3 "-" "SED_LIBRARY=$V"
cat $O/c4/ab.jsonl
echo finished
