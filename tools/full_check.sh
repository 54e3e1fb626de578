#!/bin/bash
# Full GPU suite, then the c4 bench line and a kernel trace -> gpurun_out/$TAG/
set -e
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_bench.json 2> $O/kt_bench.log
for w in c3 c2 c5; do
  timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline >> $O/bench_other.jsonl 2>> $O/bench.log
done
