#!/bin/bash
set -e
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tools/ab2.sh r03d 3 tools/ab_libs/libsed_base.so tools/ab_libs/libsed_tb1.so tools/ab_libs/libsed_h32.so
for w in iupac timing; do
  timeout -k 10 200 python3 bench.py --workload $w --traffic none --no-cpu-baseline >> $O/bench_f64.jsonl 2>> $O/bench.log
  SED_LIBRARY=$PWD/tools/ab_libs/libsed_base.so timeout -k 10 200 python3 bench.py --workload $w --traffic none --no-cpu-baseline >> $O/bench_f64_base.jsonl 2>> $O/bench.log
done
