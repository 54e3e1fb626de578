#!/bin/bash
# Round 6 step 32: c4 in 2 parts (default) against 3 and 4 parts with the traceback's own translation unit
set -e
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s32}/c4 3 "-" "SED_CK_HALVES=3" "SED_CK_HALVES=4"
cat gpurun_out/${1:-r06s32}/c4/ab.jsonl
echo finished
