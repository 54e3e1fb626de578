#!/bin/bash
# Round 5, step 13: order-independent per-call cost plans and the batched-search host path: shim/error GPU tests,
# timing.py's per-call breakdown, the caller paths
set -e
O=gpurun_out/${1:-r05s13}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_shim_gpu.py tests/test_errors_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_shim.log 2>&1
tail -1 $O/tests_shim.log
timeout -k 10 300 python3 tools/timing_breakdown.py $O/timing_breakdown.txt
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
cat $O/caller_paths.txt
