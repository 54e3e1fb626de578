#!/bin/bash
# libsed.so variants for interleaved A/Bs: the checkpoint traceback's waves at issue priority 1 and 3 (SED_CKTB_PRIO)
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for p in 1 3; do
  make -s OBJ=sed_kernels_p$p.o OUT=../../tools/ab_libs/libsed_p$p.so EXTRA="-DSED_CKTB_PRIO=$p" ../../tools/ab_libs/libsed_p$p.so
done
