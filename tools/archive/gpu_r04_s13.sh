#!/bin/bash
# Round 4: SPLIT consumer re-reads the feeder's ready count only when it is used up: the SPLIT tests, then config 2
# against the previous build, 3 interleaved rounds
set -e
O=gpurun_out/${1:-r04s13}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -k "split or stripe_parallel or config2 or g3 or handoff" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="--workload c2" timeout -k 10 400 bash tools/ab2.sh ${1:-r04s13}/c2 3 tools/ab_libs/libsed_prev.so rna-sequence-diff-patch_amd/libsed.so
cat $O/c2/ab.jsonl
