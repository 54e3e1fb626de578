#!/bin/bash
# Round 5, step 15: the checkpoint traceback's waves at issue priority 1 and 3 (s_setprio; SED_CKTB_PRIO builds)
# against the default 0, c4 at 2 parts; CK tests on the priority-3 build
set -e
O=gpurun_out/${1:-r05s15}
mkdir -p $O
export TMPDIR=/tmp
P1=SED_LIBRARY=$PWD/tools/ab_libs/libsed_p1.so
P3=SED_LIBRARY=$PWD/tools/ab_libs/libsed_p3.so
env $P3 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py -m gpu -x -v -k "checkpoint or headline" --timeout 300 --timeout-method thread > $O/tests_p3.log 2>&1
tail -1 $O/tests_p3.log
bash tools/ab_env.sh ${1:-r05s15} 3 "-" "$P1" "$P3"
cat $O/ab.jsonl
env $P3 timeout -k 10 200 python3 tools/c4_timeline.py 10 > $O/timeline_p3.txt 2>&1
head -8 $O/timeline_p3.txt
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
cat $O/caller_paths.txt
