#!/bin/bash
# libsed.so variants for interleaved A/Bs: the checkpoint traceback compiled for 6 and 8 waves per SIMD
# (SED_CKTB_WAVES; the default build leaves the register budget to the compiler: 90 VGPRs at R = 16, 5 waves)
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for w in 6 8; do
  make -s OBJ=sed_kernels_w$w.o CKTB_OBJ=sed_cktb_w$w.o OUT=../../tools/ab_libs/libsed_w$w.so EXTRA="-DSED_CKTB_WAVES=$w" ../../tools/ab_libs/libsed_w$w.so
done
