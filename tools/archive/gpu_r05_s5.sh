#!/bin/bash
# Round 5, step 5: the quarter-band traceback (sed_traceback_ckq_kernel, default at R = 16): route/parity tests, then an
# interleaved A/B against the lane-per-row sweep, alone (1 part) and in the default 2 parts
set -e
O=gpurun_out/${1:-r05s5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
bash tools/ab_env.sh ${1:-r05s5} 2 "SED_CK_REPLAY=0" "-" "SED_CK_REPLAY=0 SED_CK_HALVES=1" "SED_CK_HALVES=1"
cat $O/ab.jsonl
