#!/bin/bash
# Round 4: a 4-rank gloo rehearsal of the multi-GPU bench path on one GPU (4 shards of 8192 pairs, the gather and
# rank 0's verification of all 32 768 scripts), timed end to end
set -e
O=gpurun_out/${1:-r04s8}
mkdir -p $O
export TMPDIR=/tmp
start=$(date +%s)
timeout -k 10 500 python3 bench.py --gpus 4 --dist-backend gloo --traffic none --no-cpu-baseline > $O/dist4_c4_gloo.json 2> $O/dist4.log
echo "wall $(( $(date +%s) - start )) s" | tee $O/dist4_wall.txt
tail -4 $O/dist4.log
python3 -c "import json; d=json.loads(open('$O/dist4_c4_gloo.json').read().strip().split(chr(10))[-1]); print({k: d.get(k) for k in ('value','ms_per_step','n_gpus','script_valid_rate','script_exact_rate','verified_on_rank0')})"
