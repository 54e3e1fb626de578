#!/bin/bash
# Round 6 step 11: every walk zeroes its pair's script padding before it walks (was after): the route, parity and
# fuzz tests, then c3 / timing / c4 A/B against no zeroing (libsed_pz0.so)
set -e
O=gpurun_out/${1:-r06s11}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="--workload c3" bash tools/ab_env.sh ${1:-r06s11}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
AB_ARGS="--workload timing" bash tools/ab_env.sh ${1:-r06s11}/timing 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s11}/c4 2 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
cat $O/c3/ab.jsonl $O/timing/ab.jsonl $O/c4/ab.jsonl
echo finished
