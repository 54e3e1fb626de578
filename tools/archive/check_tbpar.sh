#!/bin/bash
# Stripe-parallel traceback: its test, the G3 / parity / shim suites, and a c2 A/B against the one-chain walk
set -e
O=gpurun_out/${1:-tbpar}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py tests/test_shim_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  SED_TBPAR=0 timeout -k 10 200 python3 bench.py --workload c2 --no-cpu-baseline --traffic none >> $O/c2_chain.jsonl 2>> $O/log
  SED_TBPAR=1 timeout -k 10 200 python3 bench.py --workload c2 --no-cpu-baseline --traffic none >> $O/c2_par.jsonl 2>> $O/log
done
