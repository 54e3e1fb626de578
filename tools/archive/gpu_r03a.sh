#!/bin/bash
# Round 3, first GPU call: dot distance microbenchmark, the GPU tests, the default bench line (with the new
# SQ issue pass and 8(d) roofline), and the self-launched 2-rank gloo rehearsal -> gpurun_out/$TAG/
set -e
TAG=${1:-r03a}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/ubench/dot_dist > $O/ubench_dot_dist.txt 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 > $O/dist2_c4.json 2> $O/dist2_c4.log
timeout -k 10 200 python3 bench.py --workload c3 --traffic none --no-cpu-baseline >> $O/bench_other.jsonl 2>> $O/bench.log
timeout -k 10 200 python3 bench.py --workload iupac --traffic none --no-cpu-baseline >> $O/bench_other.jsonl 2>> $O/bench.log
