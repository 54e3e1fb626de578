#!/bin/bash
# Does running two halves of the config-4 shard concurrently beat one 8192-pair batch?  (one GPU)
set -e
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
B="--steps 10 --warmup 2 --no-cpu-baseline --traffic none"
timeout -k 10 200 python3 bench.py $B > $O/one_8192.json 2> $O/one_8192.log
timeout -k 10 200 python3 bench.py $B --pairs 16384 > $O/one_16384.json 2> $O/one_16384.log
timeout -k 10 300 python3 bench.py $B --gpus 2 --dist-backend gloo --pairs 4096 > $O/two_4096.json 2> $O/two_4096.log
timeout -k 10 300 python3 bench.py $B --gpus 2 --dist-backend gloo > $O/two_8192.json 2> $O/two_8192.log
for f in one_8192 one_16384 two_4096 two_8192; do
  python3 -c "
import json,re
t=open('$O/$f.json').read(); d=json.loads(t[t.index('{\"metric'):].splitlines()[0])
print(json.dumps({'run':'$f','n_gpus':d['n_gpus'],'pairs':d['config']['pairs_per_gpu'],'value':d['value'],'ms_per_step':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d.get('traceback_ms'),'valid':d.get('script_valid_rate')}))" >> $O/summary.jsonl
done
cat $O/summary.jsonl
