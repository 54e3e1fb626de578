#!/bin/bash
# round 3, session 2: pipelined lane batches on two streams: tests, then c5 / c5n A/B SED_ALT_DP=0/1
set -e
O=gpurun_out/r03s5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_routes.py -m gpu -x -v --timeout 200 --timeout-method thread -k "pipelined or lane" > $O/tests_lane.log 2>&1
tail -3 $O/tests_lane.log
for w in c5 c5n; do
  for r in 1 2 3; do
    for a in 0 1; do
      SED_ALT_DP=$a timeout -k 10 120 python3 bench.py --workload $w --steps 200 --warmup 5 --no-cpu-baseline --traffic none > $O/x.json 2>> $O/x.log
      python3 -c "import json; d=json.load(open('$O/x.json')); print(json.dumps({'w':'$w','alt':$a,'value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'exact':d.get('dist_exact_rate')}))" >> $O/ab.jsonl
    done
  done
done
cat $O/ab.jsonl
