#!/bin/bash
# select-free hold: per-step dumps of visit 2 on the failing pair (both debug builds); A/B of the current build
# against the measured 3-part build (traceback kernel code moved around the VHOLD switch)
set -e
O=gpurun_out/r03dbg2
mkdir -p $O
export TMPDIR=/tmp
for L in libsed_dbg0 libsed_dbg1; do
  SED_LIBRARY=$PWD/tools/ab_libs/$L.so timeout -k 10 120 python3 -u tools/diag_vhold_dump.py >> $O/dumps.jsonl 2>> $O/dumps.err
done
SED_CK_HALVES=2 tools/ab2.sh r03dbg2_ab 3 tools/ab_libs/libsed_halves.so tools/ab_libs/libsed_cur.so
cat gpurun_out/r03dbg2_ab/ab.jsonl
