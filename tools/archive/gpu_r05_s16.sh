#!/bin/bash
# Round 5, step 16: checkpoint traceback at priority 1 now default (against 0), and the per-cell-code traceback at
# priority 1 for the pipelined workloads (c3, iupac, timing)
set -e
O=gpurun_out/${1:-r05s16}
mkdir -p $O
export TMPDIR=/tmp
CK0=SED_LIBRARY=$PWD/tools/ab_libs/libsed_ck0.so
TP1=SED_LIBRARY=$PWD/tools/ab_libs/libsed_tp1.so
bash tools/ab_env.sh ${1:-r05s16}/c4 3 "-" "$CK0" "SED_CK_HALVES=3" "SED_CK_HALVES=4"
for w in c3 timing iupac; do
  AB_ARGS="--workload $w" bash tools/ab_env.sh ${1:-r05s16}/$w 2 "-" "$TP1"
done
cat $O/*/ab.jsonl
