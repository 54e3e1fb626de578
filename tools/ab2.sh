#!/bin/bash
# Interleaved A/B of libsed builds: tools/ab2.sh TAG ROUNDS lib1.so lib2.so ... (paths relative to the repo; bench args
# in $AB_ARGS, default the c4 bench).  No PMC passes, no CPU legs.  -> gpurun_out/TAG/ab.jsonl
set -e
TAG=$1; N=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 $N); do
  for L in "$@"; do
    SED_LIBRARY=$PWD/$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --traffic none ${AB_ARGS} > $O/ab.json 2>> $O/ab.log
    python3 -c "import json; d=json.load(open('$O/ab.json')); print(json.dumps({'lib':'$L','round':$r,'value':d['value'],'dp_ms':d['roofline'].get('kernel_ms_per_step', d['roofline'].get('kernel_ms')),'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate'),'tb_ms':d.get('traceback_ms'),'step_ms':d['ms_per_step']}))" >> $O/ab.jsonl
  done
done
