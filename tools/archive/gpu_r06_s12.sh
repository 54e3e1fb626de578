#!/bin/bash
# Round 6 step 12: two-chunk windows in the checkpoint traceback (SED_CKTB_NW=12): the route, parity and fuzz tests,
# the SQ pass of the c4 kernels, then c4 A/B against one-chunk windows (libsed_nw8.so) and the previous build
set -e
O=$PWD/gpurun_out/${1:-r06s12}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
for v in def head; do
  if [ $v = def ]; then EV=""; else EV="SED_LIBRARY=$PWD/tools/ab_libs/libsed_$v.so"; fi
  env $EV timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -d $O/sq_$v -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_$v.json 2> $O/sq_$v.log
done
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s12}/c4 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_head.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_nw8.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_w5.so"
cat $O/c4/ab.jsonl
echo finished
