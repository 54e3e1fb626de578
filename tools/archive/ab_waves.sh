#!/bin/bash
# A/B: CK forward at 4 / 5 / 6 waves per SIMD (tools/ab_libs/libsed_w{4,5,6}.so, built by tools/ab_libs/build.sh),
# interleaved rounds of the c4 bench -> gpurun_out/$TAG/w*.jsonl
set -e
O=gpurun_out/${1:-abw}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for w in 4 5 6; do
    SED_LIBRARY=$PWD/tools/ab_libs/libsed_w$w.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic none --steps 20 >> $O/w$w.jsonl 2>> $O/log
  done
done
