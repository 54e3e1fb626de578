#!/bin/bash
# round 3, session 2: alternating DP streams for pipelined dynamic-CHAIN batches (config 3): route tests, then
# c3 A/B SED_ALT_DP=0/1 (3 interleaved rounds)
set -e
O=gpurun_out/r03s4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "chain" > $O/tests_chain.log 2>&1
tail -3 $O/tests_chain.log
for r in 1 2 3; do
  for a in 0 1; do
    SED_ALT_DP=$a timeout -k 10 200 python3 bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline --traffic none > $O/c3.json 2>> $O/c3.log
    python3 -c "import json; d=json.load(open('$O/c3.json')); print(json.dumps({'alt':$a,'value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d.get('traceback_ms'),'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate')}))" >> $O/c3_ab.jsonl
  done
done
cat $O/c3_ab.jsonl
