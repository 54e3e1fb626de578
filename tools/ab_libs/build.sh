#!/bin/bash
# libsed.so variants for interleaved A/Bs (tools/ab2.sh): the CK forward kernel's groups per chunk-loop iteration
# (SED_CK_GUNROLL, default 2) at 4 and 8
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for u in 4 8; do
  make -s OBJ=sed_kernels_u$u.o CKTB_OBJ=sed_cktb_u$u.o OUT=../../tools/ab_libs/libsed_u$u.so EXTRA="-DSED_CK_GUNROLL=$u" ../../tools/ab_libs/libsed_u$u.so
done
