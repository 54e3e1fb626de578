#!/bin/bash
# Round 6 step 29: the checkpoint traceback (own translation unit, 70 VGPRs: up to 7 waves per SIMD) against the same
# kernel compiled for 8 waves (SED_CKTB_WAVES=8: 64 VGPRs, 8-20 bytes of scratch), c4
set -e
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s29}/c4 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_w8.so"
cat gpurun_out/${1:-r06s29}/c4/ab.jsonl
echo finished
