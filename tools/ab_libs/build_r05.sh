#!/bin/bash
# libsed.so variants for round 5's A/Bs: the replay traceback's wave priority (SED_CKR_PRIO)
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for p in 3; do
  make -s OBJ=sed_kernels_p$p.o OUT=../../tools/ab_libs/libsed_prio$p.so EXTRA="-DSED_CKR_PRIO=$p" ../../tools/ab_libs/libsed_prio$p.so
done
