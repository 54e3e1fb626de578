#!/bin/bash
# CK GPU tests, bench line, kernel trace and the FETCH/WRITE passes -> gpurun_out/$TAG/
set -e
O=gpurun_out/${1:-cktr}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or g3 or ladder or g8" > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/fetch_bench.json 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/write -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/write_bench.json 2>&1
