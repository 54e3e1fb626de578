#!/bin/bash
# Kernel-variant sweep on the GPU box: each line runs bench.py with one library / rows-per-lane.
set -e
out=gpurun_out/sweep.jsonl
: > $out
for cfg in "libsed.so 16" "libsed_w6.so 16" "libsed_w6.so 8"; do
  set -- $cfg
  SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --rows-per-lane $2 > gpurun_out/sw.json 2> gpurun_out/sw.log
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sw.json')); print(json.dumps({'lib':'$1','R':$2,'value':d['value'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d['traceback_ms'],'valid':d['script_valid_rate']}))" >> $out
done
