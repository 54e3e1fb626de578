#!/bin/bash
# Workload / rows-per-lane sweep on the GPU box -> gpurun_out/sweep.jsonl
set -e
out=gpurun_out/sweep.jsonl
: > $out
run() {
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > gpurun_out/sw.json 2> gpurun_out/sw.log
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/sw.json'))
print(json.dumps({'args': sys.argv[1:], 'value': d['value'], 'ms_step': d['ms_per_step'], 'dp_ms': d['roofline']['kernel_ms'],
 'tb_ms': d['traceback_ms'], 'R': d['config']['rows_per_lane'], 'mode': d['config']['mode'], 'valid': d.get('script_valid_rate'),
 'valu_frac': (d['valu'] or {}).get('frac')}))" "$@" >> $out
}
for spec in "$@"; do
  run $spec
done
