#!/bin/bash
# SPLIT hand-off wait before the group's stores: SPLIT parity tests, then c2 / c2-shape A/B against the T1 build
set -e
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "split or config2 or g3 or G3" > $O/tests.log 2>&1
AB_ARGS="--workload c2 --steps 200 --warmup 10" tools/ab2.sh r03p 3 tools/ab_libs/libsed_t1.so tools/ab_libs/libsed_spw.so
AB_ARGS="--workload c2 --steps 200 --warmup 10 --shape 4096x1024" tools/ab2.sh r03p_s 2 tools/ab_libs/libsed_t1.so tools/ab_libs/libsed_spw.so
cat $O/ab.jsonl gpurun_out/r03p_s/ab.jsonl
