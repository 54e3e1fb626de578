#!/bin/bash
# Round 6 step 25: the checkpoint traceback's wave priority after the two-chunk windows: 1 (default) against 0 and 2
set -e
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s25}/c4 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_tp0.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_tp2.so"
cat gpurun_out/${1:-r06s25}/c4/ab.jsonl
echo finished
