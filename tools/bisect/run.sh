#!/bin/bash
O=gpurun_out/bisect; mkdir -p $O
SED_LIBRARY=$PWD/tools/bisect/libsed_d111.so timeout -k 10 120 python -u tools/bisect/dump.py d111 > $O/d111.log 2>&1 || exit $?
SED_LIBRARY=$PWD/tools/bisect/libsed_n111.so timeout -k 10 250 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "config3_route or checkpoint or chain or g3 or g8" > $O/n111.log 2>&1
rc=$?; echo "n111 rc=$rc $(tail -1 $O/n111.log)"; exit $rc
