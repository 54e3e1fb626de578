#!/bin/bash
# round 4 step 15: SPLIT checkpoint forward hands off lane 63's row checkpoints (no per-step collection): split and
# checkpoint tests, then a config-2 A/B against the previous build
set -e
O=gpurun_out/r04s15; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu \
  -k "split or g3 or checkpoint or stripe_parallel" > $O/tests.log 2>&1
tail -1 $O/tests.log
AB_ARGS="--workload c2 --steps 200 --warmup 20" timeout -k 10 600 bash tools/ab2.sh r04s15 4 tools/ab_libs/libsed_prev.so rna-sequence-diff-patch_amd/libsed.so
