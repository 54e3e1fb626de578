#!/bin/bash
# Interleaved A/B of two libsed builds: tools/ab.sh libA.so libB.so [rounds]  (bench args in $AB_ARGS, default c4)
set -e
A=$1; B=$2; N=${3:-3}
out=gpurun_out/ab.jsonl
: > $out
for r in $(seq 1 $N); do
  for L in $A $B; do
    SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.log
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'lib':'$L','round':$r,'value':d['value'],'dp_ms':d['roofline']['kernel_ms'],'valid':d.get('script_valid_rate'),'tb_ms':d.get('traceback_ms'),'step_ms':d['ms_per_step']}))" >> $out
  done
done
