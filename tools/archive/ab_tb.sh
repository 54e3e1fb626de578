#!/bin/bash
# A/B of two libsed builds on step time and traceback time (pipelined and not): tools/ab_tb.sh libA libB [rounds]
set -e
A=$1; B=$2; N=${3:-2}
out=gpurun_out/ab_tb.jsonl
: > $out
for r in $(seq 1 $N); do
  for L in $A $B; do
    for P in "" "--no-pipeline"; do
      SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$L timeout -k 10 200 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline $P ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.log
      python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'lib':'$L','pipe':'$P'=='','value':d['value'],'ms_step':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d['traceback_ms'],'valid':d.get('script_valid_rate')}))" >> $out
    done
  done
done
