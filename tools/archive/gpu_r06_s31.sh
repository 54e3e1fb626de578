#!/bin/bash
# Round 6 step 31: the wide ladder with its row-0 jump folded into the DPP move (4-bit rung field, one jump row in 8) for the CHAIN kernel's ladder dot keys: the
# route, parity and fuzz GPU tests, then config 3 A/B against the previous build
set -e
O=$PWD/gpurun_out/${1:-r06s31}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="--workload c3 --steps 20" bash tools/ab_env.sh ${1:-r06s31}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_wide.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_head.so"
cat $O/c3/ab.jsonl
echo finished
