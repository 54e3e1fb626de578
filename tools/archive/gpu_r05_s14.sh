#!/bin/bash
# Round 5, step 14: pipelined checkpoint parts (SED_CK_PIPELINE=1: each part's traceback on the traceback stream
# behind its forward, three checkpoint buffers): CK tests under it, c4 A/B against the default stagger
set -e
O=gpurun_out/${1:-r05s14}
mkdir -p $O
export TMPDIR=/tmp
SED_CK_PIPELINE=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py -m gpu -v -k "checkpoint or ck or headline" --timeout 300 --timeout-method thread > $O/tests_pipe.log 2>&1 || true
tail -1 $O/tests_pipe.log
bash tools/ab_env.sh ${1:-r05s14} 2 "-" "SED_CK_PIPELINE=1" "SED_CK_PIPELINE=1 SED_CK_HALVES=3" "SED_CK_PIPELINE=1 SED_CK_HALVES=1"
cat $O/ab.jsonl
SED_CK_PIPELINE=1 timeout -k 10 200 python3 tools/c4_timeline.py 10 > $O/timeline_pipe.txt 2>&1
head -12 $O/timeline_pipe.txt
