#!/bin/bash
# Builds traceback variants of libsed.so (compile-time switches) into tools/bisect/
set -e
cd "$(dirname "$0")/../../rna-sequence-diff-patch_amd/csrc"
for v in "d111 -DSED_TB_DEBUG" "n111 " ; do
  set -- $v; tag=$1; shift
  make -s OBJ=sed_kernels_$tag.o OUT=../../tools/bisect/libsed_$tag.so EXTRA="$*" ../../tools/bisect/libsed_$tag.so
done
