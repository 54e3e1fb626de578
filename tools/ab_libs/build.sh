#!/bin/bash
# libsed.so variants with the CK forward kernel's waves-per-SIMD target (SED_CK_WAVES) at 4, 5 and 6
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for w in 4 5 6; do
  make -s OBJ=sed_kernels_w$w.o OUT=../../tools/ab_libs/libsed_w$w.so EXTRA="-DSED_CK_WAVES=$w" ../../tools/ab_libs/libsed_w$w.so
done
