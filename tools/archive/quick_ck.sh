#!/bin/bash
# Quick loop for the checkpoint path: its GPU tests, the c4 bench line, and a kernel trace -> gpurun_out/$TAG/
set -e
TAG=${1:-ck}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or chain or g3 or g8" > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_bench.json 2> $O/kt_bench.log
