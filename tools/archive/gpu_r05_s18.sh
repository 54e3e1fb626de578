#!/bin/bash
# Round 5, step 18: with the checkpoint traceback at issue priority 1, its occupancy again: 6 and 8 waves per SIMD
# (80 / 64 VGPRs) against the compiler's 90 (5 waves)
set -e
O=gpurun_out/${1:-r05s18}
mkdir -p $O
export TMPDIR=/tmp
W6=SED_LIBRARY=$PWD/tools/ab_libs/libsed_w6.so
W8=SED_LIBRARY=$PWD/tools/ab_libs/libsed_w8.so
bash tools/ab_env.sh ${1:-r05s18} 3 "-" "$W6" "$W8"
cat $O/ab.jsonl
