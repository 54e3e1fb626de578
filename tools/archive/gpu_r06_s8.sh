#!/bin/bash
# Round 6 step 8: does the per-lane padding zeroing (zero_script_tail) cost config 3 / timing?  Interleaved A/B of
# the default build against SED_PAD_ZERO=0 (libsed_pz0.so), 3 rounds each
set -e
O=gpurun_out/${1:-r06s8}
mkdir -p $O
export TMPDIR=/tmp
AB_ARGS="--workload c3" bash tools/ab_env.sh ${1:-r06s8}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
AB_ARGS="--workload timing" bash tools/ab_env.sh ${1:-r06s8}/timing 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
cat $O/c3/ab.jsonl $O/timing/ab.jsonl
echo finished
