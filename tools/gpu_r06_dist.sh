#!/bin/bash
# Round 6: fp64 batches of many long pairs (SPLIT gate), then the 8-rank launch + gather rehearsal on one
# GPU (gloo; self-launched ranks, rank 0 verifies every gathered pair) for c4 (512 pairs per rank) and c5
set -e
O=gpurun_out/${1:-r06dist}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/fp64_split_batch.py $O/fp64_split_batch.txt > $O/fp64_split_batch.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 8 --dist-backend gloo --pairs 512 --steps 5 --warmup 1 --traffic none --no-cpu-baseline > $O/dist8_c4_gloo.json 2> $O/dist8_c4.log
timeout -k 10 300 python3 bench.py --gpus 8 --dist-backend gloo --workload c5 --steps 5 --warmup 1 --traffic none --no-cpu-baseline > $O/dist8_c5_gloo.json 2> $O/dist8_c5.log
python3 -c "
import json
for f in ('dist8_c4_gloo', 'dist8_c5_gloo'):
    d = json.load(open('$O/%s.json' % f))
    print(f, d['n_gpus'], d['ms_per_step'], d.get('gather_ms'), d.get('script_valid_rate'), d.get('script_exact_rate'), d.get('dist_exact_rate'), d.get('verified_on_rank0', {}).get('pairs'), d.get('shards'))"
echo finished
