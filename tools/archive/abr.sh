#!/bin/bash
# A/B of (library, bench args, env) variants, interleaved: tools/abr.sh ROUNDS "lib|args|VAR=val ..." ...
set -e
N=$1; shift
out=gpurun_out/abr.jsonl
for r in $(seq 1 $N); do
  for spec in "$@"; do
    IFS='|' read -r L A E <<< "$spec"
    env SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$L $E timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline $A > gpurun_out/ab.json 2> gpurun_out/ab.log
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'lib':'$L','args':'$A','env':'$E','round':$r,'value':d['value'],'dp_ms':d['roofline']['kernel_ms'],'valid':d.get('script_valid_rate'),'tb_ms':d.get('traceback_ms'),'step_ms':d['ms_per_step'],'R':d['config']['rows_per_lane']}))" >> $out
  done
done
