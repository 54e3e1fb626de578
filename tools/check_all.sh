#!/bin/bash
# Full GPU suite, every workload's bench line (c4 default, c3, c2, c5, c5n) and a config-2 kernel trace
set -e
O=gpurun_out/${1:-all}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic none > $O/bench_c4.json 2> $O/bench.log
for w in c3 c2 c5 c5n; do
  timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline --traffic none >> $O/bench_other.jsonl 2>> $O/bench.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --workload c2 --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c2.json 2> $O/kt_c2.log
