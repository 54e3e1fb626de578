#!/bin/bash
# Round 5, step 2: the unchanged callers' process model (fork after HIP init) and timing.py's per-call loop:
# parent-served children, then the engine-worker children of round 4 for comparison; the shim GPU tests
set -e
O=gpurun_out/${1:-r05s2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_shim_gpu.py tests/test_errors_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_shim.log 2>&1
tail -1 $O/tests_shim.log
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
SED_FORK_ENGINE=worker timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths_worker.json > $O/caller_paths_worker.txt 2>&1
cat $O/caller_paths.txt $O/caller_paths_worker.txt
