#!/bin/bash
# Round 5, step 17: DP-side issue priorities: SPLIT's stripe waves at 2 (config 2), the fp64 DP at 1 (iupac, timing)
set -e
O=gpurun_out/${1:-r05s17}
mkdir -p $O
export TMPDIR=/tmp
SP2=SED_LIBRARY=$PWD/tools/ab_libs/libsed_sp2.so
FP1=SED_LIBRARY=$PWD/tools/ab_libs/libsed_fp1.so
AB_ARGS="--workload c2 --steps 100 --warmup 10" bash tools/ab_env.sh ${1:-r05s17}/c2 3 "-" "$SP2"
for w in iupac timing; do
  AB_ARGS="--workload $w" bash tools/ab_env.sh ${1:-r05s17}/$w 3 "-" "$FP1"
done
cat $O/*/ab.jsonl
