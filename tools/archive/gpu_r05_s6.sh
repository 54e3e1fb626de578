#!/bin/bash
# Round 5, step 6: the replay traceback (few long-running waves) pipelined beside the next run's forward
# (SED_CK_PIPELINE=1, one part: run k's traceback on the traceback stream while run k+1's forward runs)
set -e
O=gpurun_out/${1:-r05s6}
mkdir -p $O
export TMPDIR=/tmp
P3=SED_LIBRARY=$PWD/tools/ab_libs/libsed_prio3.so
bash tools/ab_env.sh ${1:-r05s6} 2 "SED_CK_REPLAY=0" "SED_CK_REPLAY=1 SED_CK_HALVES=1 SED_CK_PIPELINE=1" "$P3 SED_CK_REPLAY=1 SED_CK_HALVES=1 SED_CK_PIPELINE=1" "SED_CK_REPLAY=0 SED_CK_HALVES=1 SED_CK_PIPELINE=1"
cat $O/ab.jsonl
