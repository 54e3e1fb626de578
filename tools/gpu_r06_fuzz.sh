#!/bin/bash
# Round 6: longer runs of the route fuzz (padding checked too) and the module fuzz on the final code
set -e
O=gpurun_out/${1:-r06fuzz}
mkdir -p $O
export TMPDIR=/tmp
SED_FUZZ_SECONDS=${2:-240} SED_FUZZ_SEED=${3:-606000} timeout -k 10 500 python3 -u -m pytest tests/test_fuzz_gpu.py -m gpu -x -v -s --timeout 480 --timeout-method thread -k route > $O/route_fuzz.log 2>&1
tail -3 $O/route_fuzz.log
SED_FUZZ_MODULE_SECONDS=${4:-120} SED_FUZZ_SEED=${3:-606000} timeout -k 10 300 python3 -u -m pytest tests/test_fuzz_gpu.py -m gpu -x -v -s --timeout 280 --timeout-method thread -k module > $O/module_fuzz.log 2>&1
tail -3 $O/module_fuzz.log
echo finished
