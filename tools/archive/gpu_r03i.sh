#!/bin/bash
set -e
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tools/ab2.sh r03i 3 tools/ab_libs/libsed_base.so tools/ab_libs/libsed_t1.so
for sh in 256x4096 512x4096 1024x4096 2048x4096 4096x4096 4096x1024; do
  timeout -k 10 120 python3 bench.py --workload c2 --shape $sh --steps 100 --warmup 5 --no-cpu-baseline --traffic none >> $O/c2_shapes.jsonl 2>> $O/c2.log
done
