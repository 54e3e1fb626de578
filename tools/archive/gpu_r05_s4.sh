#!/bin/bash
# Round 5, step 4: the replay traceback's schedule -- wave priority and parts, against the lane-per-row sweep
set -e
O=gpurun_out/${1:-r05s4}
mkdir -p $O
export TMPDIR=/tmp
P3=SED_LIBRARY=$PWD/tools/ab_libs/libsed_prio3.so
bash tools/ab_env.sh ${1:-r05s4} 2 "SED_CK_REPLAY=0" "-" "$P3" "$P3 SED_CK_HALVES=4" "$P3 SED_CK_HALVES=1" "SED_CK_REPLAY=0 SED_CK_HALVES=1"
cat $O/ab.jsonl
env $P3 timeout -k 10 200 python3 tools/c4_timeline.py 10 > $O/timeline_prio3.txt 2>&1
SED_CK_REPLAY=0 timeout -k 10 200 python3 tools/c4_timeline.py 10 > $O/timeline_old.txt 2>&1
tail -5 $O/timeline_prio3.txt $O/timeline_old.txt
