#!/bin/bash
# Round 6 step 28: private arrays kept out of vector registers in every kernel (tools/ab_libs/libsed_pa.so) against the
# default build, on the fp64 workloads (iupac, timing) and config 3
set -e
AB_ARGS="--workload iupac" bash tools/ab_env.sh ${1:-r06s28}/iupac 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pa.so"
AB_ARGS="--workload timing" bash tools/ab_env.sh ${1:-r06s28}/timing 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pa.so"
AB_ARGS="--workload c3" bash tools/ab_env.sh ${1:-r06s28}/c3 2 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pa.so"
cat gpurun_out/${1:-r06s28}/*/ab.jsonl
echo finished
