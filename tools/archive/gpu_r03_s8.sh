#!/bin/bash
# round 3, session 2: checkpoint parts 2 vs 3 on c4 (default bench shape, 20 steps, 4 interleaved rounds)
set -e
O=gpurun_out/r03s8
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3 4; do
  for V in "SED_CK_HALVES=2" "SED_CK_HALVES=3"; do
    env $V timeout -k 10 200 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --traffic none > $O/ab.json 2>> $O/ab.log
    python3 -c "import json; d=json.load(open('$O/ab.json')); print(json.dumps({'env':'$V','round':$r,'value':d['value'],'dp_ms':d['roofline']['kernel_ms'],'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate'),'tb_ms':d.get('traceback_ms'),'step_ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
