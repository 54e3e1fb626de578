#!/bin/bash
# GPU parity tests, then every bench workload once without the CPU baseline -> gpurun_out/$TAG/
set -e
TAG=${1:-chk}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
shift || true
for w in ${@:-c4 c3 c2 c5 c5n iupac}; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline >> $O/bench.jsonl 2>> $O/bench.log
done
for w in c4 c3; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-script >> $O/bench_noscript.jsonl 2>> $O/bench.log
done
