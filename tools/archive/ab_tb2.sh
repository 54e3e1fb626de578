#!/bin/bash
# Traceback A/B: standalone traceback time (--no-pipeline) and step time on c2 / c3 / c4
set -e
A=$1; B=$2
out=gpurun_out/ab_tb2.jsonl
: > $out
for W in c2 c3 c4; do
  for L in $A $B; do
    for P in "" "--no-pipeline"; do
      SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$L timeout -k 10 200 python3 bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline $P > gpurun_out/ab.json 2> gpurun_out/ab.log
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'w':'$W','lib':'$L','pipe':'$P'=='','ms_step':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d['traceback_ms'],'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate')}))" >> $out
    done
  done
done
