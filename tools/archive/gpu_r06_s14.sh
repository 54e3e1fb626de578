#!/bin/bash
# Round 6 step 14: config 3 on checkpoints (SED_OPT_TB = 2) against its per-cell-code CHAIN route after the two-chunk
# traceback windows, 3 interleaved rounds at 10 steps; and config 2 (the GUI pair, checkpoint codes kernel) once
set -e
O=gpurun_out/${1:-r06s14}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for tb in 0 2; do
    timeout -k 10 200 python3 bench.py --workload c3 --tb $tb --steps 10 --warmup 2 --no-cpu-baseline --traffic none > $O/c3_tb$tb.json 2>> $O/c3.log
    python3 -c "import json; d=json.load(open('$O/c3_tb$tb.json')); print(json.dumps({'tb':$tb,'round':$r,'step_ms':d['ms_per_step'],'tb_ms':d.get('traceback_ms'),'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate')}))" >> $O/c3_ab.jsonl
  done
done
timeout -k 10 200 python3 bench.py --workload c2 --no-cpu-baseline --traffic none > $O/c2.json 2> $O/c2.log
cat $O/c3_ab.jsonl
python3 -c "import json; d=json.load(open('$O/c2.json')); print({k: d.get(k) for k in ('ms_per_step','script_valid_rate','script_exact_rate')})"
echo finished
