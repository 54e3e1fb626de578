#!/bin/bash
# Full GPU suite, then the c4 and c3 bench lines -> gpurun_out/$TAG/
set -e
O=gpurun_out/${1:-c34}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic none > $O/c4.json 2> $O/bench.log
timeout -k 10 200 python3 bench.py --workload c3 --no-cpu-baseline --traffic none > $O/c3.json 2>> $O/bench.log
timeout -k 10 200 python3 bench.py --workload c3 --no-cpu-baseline --traffic none >> $O/c3.json 2>> $O/bench.log
