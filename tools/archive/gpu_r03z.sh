#!/bin/bash
# fp64 rows per lane on the timing / iupac workloads (R = 4 vs the automatic 8)
set -e
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
for A in "--workload timing --rows-per-lane 4" "--workload timing --rows-per-lane 8" "--workload iupac --rows-per-lane 4" "--workload iupac --rows-per-lane 8"; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --traffic none $A > $O/r.json 2>> $O/r.log
  python3 -c "import json; d=json.load(open('$O/r.json')); print(json.dumps({'args':'$A','value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d.get('traceback_ms'),'valid':d.get('script_valid_rate')}))" >> $O/fp64_R.jsonl
done
cat $O/fp64_R.jsonl
