#!/bin/bash
# A/B: CK forward at 6 waves/SIMD (in-tree libsed.so) vs 5 (tools/ab_libs/libsed_w5.so), interleaved
set -e
O=gpurun_out/${1:-abw}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 >> $O/w6.jsonl 2>> $O/log
  SED_LIBRARY=$PWD/tools/ab_libs/libsed_w5.so  # built with make EXTRA=-DSED_CK_WAVES=5 OUT=... timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 >> $O/w5.jsonl 2>> $O/log
done
