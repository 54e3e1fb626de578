#!/bin/bash
# Round 4: c4 with each part's traceback on its own high-priority stream (SED_CK_TBPRIO=1, since removed) against the default
# stagger: the checkpoint-parts tests under the knob, the parts timeline, 3 interleaved rounds
set -e
O=gpurun_out/${1:-r04s9}
mkdir -p $O
export TMPDIR=/tmp
SED_CK_TBPRIO=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routes.py -m gpu -k "parts_on_streams or headline" > $O/tests_tbprio.log 2>&1
tail -2 $O/tests_tbprio.log
SED_CK_TBPRIO=1 timeout -k 10 200 python3 tools/c4_timeline.py 20 > $O/timeline_tbprio.txt 2>&1
timeout -k 10 200 python3 tools/c4_timeline.py 20 > $O/timeline_default.txt 2>&1
cat $O/timeline_tbprio.txt $O/timeline_default.txt
timeout -k 10 600 bash tools/ab_env.sh ${1:-r04s9}/ab 3 - SED_CK_TBPRIO=1
cat $O/ab/ab.jsonl
