#!/bin/bash
# Round 6 step 24: config 2 at rows per lane 2 / 4 / 8, with and without the checkpoint codes (what the SPLIT
# chain's latency does with a shorter per-step chain and more stripes)
set -e
O=gpurun_out/${1:-r06s24}
mkdir -p $O
export TMPDIR=/tmp
for a in "" "--rows-per-lane 2" "--rows-per-lane 8" "--no-split-ck" "--no-split-ck --rows-per-lane 2"; do
  timeout -k 10 200 python3 bench.py --workload c2 --no-cpu-baseline --traffic none $a > $O/b.json 2>> $O/b.log
  python3 -c "import json; d=json.load(open('$O/b.json')); print(json.dumps({'args':'$a','ms':d['ms_per_step'],'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate'),'tb_ms':d.get('traceback_ms'),'R':d['config'].get('rows_per_lane'),'mode':d['config'].get('route') or d['config'].get('traceback_mode')}))" | tee -a $O/c2.jsonl
done
echo finished
