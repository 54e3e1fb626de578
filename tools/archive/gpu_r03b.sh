#!/bin/bash
set -e
TAG=${1:-r03b}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/diag_tables.py > $O/diag_tables.txt 2>&1 || true
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 > $O/dist2_c4.json 2> $O/dist2_c4.log
timeout -k 10 200 python3 bench.py --workload c3 --traffic none --no-cpu-baseline >> $O/bench_other.jsonl 2>> $O/bench.log
timeout -k 10 200 python3 bench.py --workload iupac --traffic none --no-cpu-baseline >> $O/bench_other.jsonl 2>> $O/bench.log
