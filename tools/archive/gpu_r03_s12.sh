#!/bin/bash
# round 3, session 2: every GPU test and the smoke on the final build
set -e
O=gpurun_out/r03s12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --workload c5 --traffic none --no-python-baseline --cpu-seconds 5 > $O/bench_c5.json 2> $O/bench_c5.log
cat $O/bench_c5.json | cut -c1-300
