#!/bin/bash
# SPLIT feeder wave: SPLIT tests, then c2 shapes A/B against the previous SPLIT build
set -e
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_routes.py -m gpu -x -v --timeout 120 --timeout-method thread -k "split or config2 or g3 or G3 or stripe_parallel" > $O/tests.log 2>&1
for SH in 4096x4096 4096x1024; do
  AB_ARGS="--workload c2 --steps 200 --warmup 10 --shape $SH" tools/ab2.sh r03r_$SH 2 tools/ab_libs/libsed_spb.so tools/ab_libs/libsed_feed.so
done
tail -3 $O/tests.log
cat gpurun_out/r03r_*/ab.jsonl
