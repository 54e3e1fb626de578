#!/bin/bash
# libsed.so variants for interleaved A/Bs: the per-cell-code traceback's waves at issue priority 1 (SED_TB_PRIO;
# config 3's pipelined traceback beside the next run's DP), and the checkpoint traceback back at priority 0
# (SED_CKTB_PRIO, default 1)
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
make -s OBJ=sed_kernels_tp1.o CKTB_OBJ=sed_cktb_tp1.o OUT=../../tools/ab_libs/libsed_tp1.so EXTRA="-DSED_TB_PRIO=1" ../../tools/ab_libs/libsed_tp1.so
make -s OBJ=sed_kernels_ck0.o CKTB_OBJ=sed_cktb_ck0.o OUT=../../tools/ab_libs/libsed_ck0.so EXTRA="-DSED_CKTB_PRIO=0" ../../tools/ab_libs/libsed_ck0.so
