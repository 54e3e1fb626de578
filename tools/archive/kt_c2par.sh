#!/bin/bash
# kernel trace of config 2 with the stripe-parallel traceback
set -e
O=gpurun_out/${1:-ktc2}
mkdir -p $O
export TMPDIR=/tmp
SED_TBPAR=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/b.json 2> $O/b.log
