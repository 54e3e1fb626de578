#!/bin/bash
# checkpoint batches in two halves on two streams: A/B off / joined / unjoined (c4), then c4 with halves and the oracle sample
set -e
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
tools/ab_env.sh r03w 3 "SED_CK_HALVES=0" "SED_CK_HALVES=1" "SED_CK_HALVES=2"
cat $O/ab.jsonl
SED_CK_HALVES=1 timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --traffic none --no-python-baseline --cpu-seconds 5 > $O/c4_halves.json 2> $O/c4_halves.log
python3 -c "import json; d=json.load(open('$O/c4_halves.json')); print({k: d.get(k) for k in ('value','ms_per_step','script_valid_rate','script_exact_rate')})"
