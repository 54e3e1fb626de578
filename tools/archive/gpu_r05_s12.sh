#!/bin/bash
# Round 5, step 12: the checkpoint traceback compiled for 6 and 8 waves per SIMD (80 / 64 VGPRs against the
# compiler's 90): CK tests on the 8-wave build, c4 A/B at 2 parts and 1 part
set -e
O=gpurun_out/${1:-r05s12}
mkdir -p $O
export TMPDIR=/tmp
W8=SED_LIBRARY=$PWD/tools/ab_libs/libsed_w8.so
W6=SED_LIBRARY=$PWD/tools/ab_libs/libsed_w6.so
env $W8 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v -k "checkpoint or ck or headline" --timeout 300 --timeout-method thread > $O/tests_w8.log 2>&1
tail -1 $O/tests_w8.log
bash tools/ab_env.sh ${1:-r05s12} 2 "-" "$W6" "$W8" "SED_CK_HALVES=1" "$W6 SED_CK_HALVES=1" "$W8 SED_CK_HALVES=1"
cat $O/ab.jsonl
