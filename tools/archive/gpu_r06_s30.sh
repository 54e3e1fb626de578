#!/bin/bash
# Round 6 step 30: the wide ladder (4-bit rung field, one jump row in 8) for the CHAIN kernel's ladder dot keys: the
# route, parity and fuzz GPU tests, then config 3 A/B against the previous build
set -e
O=$PWD/gpurun_out/${1:-r06s30}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="--workload c3 --steps 20" bash tools/ab_env.sh ${1:-r06s30}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_head.so"
cat $O/c3/ab.jsonl
echo finished
