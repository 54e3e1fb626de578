#!/bin/bash
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
SED_LIBRARY=$PWD/tools/ab_libs/libsed_dbg.so timeout -k 10 120 python3 -u tools/dbg_f64.py > $O/dbg_f64.txt 2>&1
SED_LIBRARY=$PWD/tools/ab_libs/libsed_tb1h32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_routes.py -m gpu -x -q --timeout 200 --timeout-method thread -k "checkpoint or dot or corrupt" > $O/tests_tb1h32.log 2>&1
echo done
