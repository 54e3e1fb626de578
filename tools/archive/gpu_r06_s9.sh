#!/bin/bash
# Round 6 step 9: the lane-per-pair walks zero their pairs' script padding as coalesced runs per wave
# (zero_script_tails_wave): the route, parity and fuzz tests, then the c3 / timing A/B against no zeroing
set -e
O=gpurun_out/${1:-r06s9}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="--workload c3" bash tools/ab_env.sh ${1:-r06s9}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
AB_ARGS="--workload timing" bash tools/ab_env.sh ${1:-r06s9}/timing 2 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
cat $O/c3/ab.jsonl $O/timing/ab.jsonl
echo finished
