#!/bin/bash
# Round 4, second GPU call: GPU suite (small-batch blob path, untimed one-shot runs, scaled lane kernel v2), per-call
# latency, host enqueue with and without timing events, c5 / c5n A/B of timing events, c4 regression line
set -e
O=gpurun_out/${1:-r04s2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 120 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
cat $O/call_latency.txt
timeout -k 10 200 python3 tools/host_overhead.py > $O/host_overhead.txt 2>&1
cat $O/host_overhead.txt
for r in 1 2; do
  for w in c5 c5n; do
    for k in 1 0; do
      timeout -k 10 300 python3 bench.py --workload $w --timing-every $k --steps 200 --warmup 20 --traffic none --no-cpu-baseline >> $O/bench_c5.jsonl 2>> $O/bench_c5.log
    done
  done
done
timeout -k 10 300 python3 bench.py --workload c5n --traffic none --no-python-baseline --cpu-seconds 3 >> $O/bench_c5.jsonl 2>> $O/bench_c5.log
timeout -k 10 300 python3 bench.py --traffic none --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.log
echo finished
