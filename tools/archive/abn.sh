#!/bin/bash
# Interleaved A/B/... of libsed builds: tools/abn.sh ROUNDS libA.so libB.so ...  (bench args in $AB_ARGS, default c4)
set -e
N=$1; shift
out=gpurun_out/abn.jsonl
for r in $(seq 1 $N); do
  for L in "$@"; do
    SED_LIBRARY=$PWD/rna-sequence-diff-patch_amd/$L timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.log
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(json.dumps({'lib':'$L','args':'${AB_ARGS}','round':$r,'value':d['value'],'dp_ms':d['roofline']['kernel_ms'],'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate'),'tb_ms':d.get('traceback_ms'),'step_ms':d['ms_per_step']}))" >> $out
  done
done
