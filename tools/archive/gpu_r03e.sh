#!/bin/bash
set -e
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/diag_f64.py > $O/diag_f64.txt 2>&1 || true
timeout -k 10 400 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or dot or g3 or corrupt or medium or routes" > $O/tests_ck.log 2>&1 || true
