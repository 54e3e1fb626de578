#!/bin/bash
# Round 5, step 11: config 3 at the bench's default step count (pipelined runs: 1/steps of an unoverlapped
# traceback), c4 default, forked wfsearch with the warm second search
set -e
O=gpurun_out/${1:-r05s11}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for w in c3 c4; do
    timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline --traffic none > $O/$w.json 2>> $O/bench.log
    python3 -c "import json; d=json.load(open('$O/$w.json')); print(json.dumps({'w':'$w','round':$r,'value':d['value'],'step_ms':d['ms_per_step'],'steps':d['steps'],'tb_ms':d.get('traceback_ms'),'busy':d['roofline'].get('kernel_ms_per_step'),'valid':d.get('script_valid_rate')}))" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
cat $O/caller_paths.txt
