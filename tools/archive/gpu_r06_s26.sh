#!/bin/bash
# Round 6 step 26: the checkpoint traceback's wave priority 1 (default) against 2 and 3, 4 interleaved rounds
set -e
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s26}/c4 4 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_tp2.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_tp3.so"
cat gpurun_out/${1:-r06s26}/c4/ab.jsonl
echo finished
