#!/bin/bash
# CHAIN plain-chunk loop: chain / route tests, c3 A/B; then the two-halves concurrency probe (tools/gpu_r03u.sh)
set -e
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "chain or dot_keys or route or ck or checkpoint" > $O/tests.log 2>&1
tail -3 $O/tests.log
AB_ARGS="--workload c3 --steps 20" tools/ab2.sh r03v_c3 3 tools/ab_libs/libsed_feed.so tools/ab_libs/libsed_pc.so
cat gpurun_out/r03v_c3/ab.jsonl
bash tools/gpu_r03u.sh
