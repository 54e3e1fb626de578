#!/bin/bash
# libsed.so variants (m0: the stripe map kernel instead of band maps) for the stripe-parallel traceback's map kernel: fewer staged columns left of each block
# (SED_TBMAP_LEFT, default 512) and shorter insert runs (SED_TBMAP_RUN, default 96) before an entry is left unknown
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
make -s OBJ=sed_kernels_m1.o CKTB_OBJ=sed_cktb_m1.o OUT=../../tools/ab_libs/libsed_m1.so EXTRA="-DSED_TBMAP_LEFT=192 -DSED_TBMAP_RUN=48" ../../tools/ab_libs/libsed_m1.so
make -s OBJ=sed_kernels_m2.o CKTB_OBJ=sed_cktb_m2.o OUT=../../tools/ab_libs/libsed_m2.so EXTRA="-DSED_TBMAP_RUN=48" ../../tools/ab_libs/libsed_m2.so
make -s OBJ=sed_kernels_m3.o CKTB_OBJ=sed_cktb_m3.o OUT=../../tools/ab_libs/libsed_m3.so EXTRA="-DSED_TBMAP_LEFT=192" ../../tools/ab_libs/libsed_m3.so
# one lane per stripe (the map before round 5's band maps)
make -s OBJ=sed_kernels_m0.o CKTB_OBJ=sed_cktb_m0.o OUT=../../tools/ab_libs/libsed_m0.so EXTRA="-DSED_TBMAP_BANDS=0" ../../tools/ab_libs/libsed_m0.so
