#!/bin/bash
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
SED_LIBRARY=$PWD/tools/ab_libs/libsed_ck2dbg.so timeout -k 10 120 python3 -u tools/dbg_ck2.py > $O/dbg_ck2.txt 2>&1
timeout -k 10 200 python3 -u tools/diag_f64.py > $O/diag_f64.txt 2>&1
echo done
