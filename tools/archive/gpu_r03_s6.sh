#!/bin/bash
# round 3, session 2: refreshed lines of the non-default workloads (pipelined by default now), kernel traces of c3 / c5
set -e
O=gpurun_out/r03s6
mkdir -p $O
export TMPDIR=/tmp
for w in c3 c2 c5 c5n iupac timing; do
  timeout -k 10 300 python3 bench.py --workload $w --traffic none --no-python-baseline --cpu-seconds 5 >> $O/bench_other.jsonl 2>> $O/bench_other.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c3 -o kt --output-format csv -- python3 bench.py --workload c3 --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c3.json 2> $O/kt_c3.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c5 -o kt --output-format csv -- python3 bench.py --workload c5 --steps 50 --warmup 2 --no-cpu-baseline --traffic none > $O/kt_c5.json 2> $O/kt_c5.log
echo finished
