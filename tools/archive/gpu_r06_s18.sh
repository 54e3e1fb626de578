#!/bin/bash
# Round 6 step 18: c4 parts on streams after the two-chunk traceback: SED_CK_HALVES = 2 (default), 1, 3, 4
set -e
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s18}/c4 3 "-" "SED_CK_HALVES=1" "SED_CK_HALVES=3" "SED_CK_HALVES=4"
cat gpurun_out/${1:-r06s18}/c4/ab.jsonl
echo finished
