#!/bin/bash
# Round-2 evidence run: full GPU suite, a 2-rank gloo rehearsal of the multi-GPU bench (ranks share the
# one GPU), the G3-scale co-optimal paths timing and the default bench line with both CPU baselines.
set -e
O=gpurun_out/${1:-r02e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo > $O/dist2_c4.json 2> $O/dist2_c4.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 2 --workload c5 --dist-backend gloo > $O/dist2_c5.json 2> $O/dist2_c5.log
timeout -k 10 300 python tools/copaths_g3.py > $O/copaths_g3.json 2> $O/copaths_g3.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.log
