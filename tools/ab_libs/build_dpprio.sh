#!/bin/bash
# libsed.so variants for interleaved A/Bs (the defaults since round 5; rebuild with 0 to compare): SPLIT's stripe waves at
# issue priority 2 (config 2), the fp64 DP's waves at
# priority 1 (iupac, timing)
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
make -s OBJ=sed_kernels_sp2.o CKTB_OBJ=sed_cktb_sp2.o OUT=../../tools/ab_libs/libsed_sp2.so EXTRA="-DSED_SPLIT_PRIO=2" ../../tools/ab_libs/libsed_sp2.so
make -s OBJ=sed_kernels_fp1.o CKTB_OBJ=sed_cktb_fp1.o OUT=../../tools/ab_libs/libsed_fp1.so EXTRA="-DSED_F64_PRIO=1" ../../tools/ab_libs/libsed_fp1.so
