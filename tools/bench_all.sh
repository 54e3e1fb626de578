#!/bin/bash
# Every bench workload once (full JSON lines, CPU baselines included) -> gpurun_out/bench_all.jsonl
set -e
out=gpurun_out/bench_all.jsonl
: > $out
for w in "$@"; do
  timeout -k 10 400 python3 bench.py --workload $w --steps ${STEPS:-10} --warmup 2 >> $out 2> gpurun_out/bench_$w.log
done
