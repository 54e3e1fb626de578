#!/bin/bash
# Round 6 step 27: the checkpoint traceback in its own translation unit, built with private arrays kept out of vector
# registers (no whole-array v_mov_b64 copies; 66-70 VGPRs instead of 96) and the top-row reads through one base
# register: the route, parity and fuzz GPU tests, the SQ pass, and c4 A/B against the previous build
set -e
O=$PWD/gpurun_out/${1:-r06s27}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -d $O/sq -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq.json 2> $O/sq.log
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s27}/c4 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_head.so"
cat $O/c4/ab.jsonl
echo finished
