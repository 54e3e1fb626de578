#!/bin/bash
# round 4 step 14: CK forward chunk loop split into unrolled (before the sink) and rolled loops: CK tests, c4 A/B
set -e
O=gpurun_out/r04s14; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu \
  -k "checkpoint or headline or dot_keys or split_checkpoint" > $O/tests.log 2>&1
AB_ARGS="" timeout -k 10 900 bash tools/ab2.sh r04s14 3 tools/ab_libs/libsed_prev.so rna-sequence-diff-patch_amd/libsed.so
