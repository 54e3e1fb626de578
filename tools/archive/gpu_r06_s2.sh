#!/bin/bash
# Round 6 step 2: the GPU suite after the ADVICE fixes (fp64 SPLIT forced over segments, R = 2 fallback, split epoch
# generations, zero-copy in-flight tracking, the fork selector thread), then fp64 many-pair SPLIT on skinny shapes
set -e
O=gpurun_out/${1:-r06s2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
SED_SPLIT_SIZES=256x2000x100,256x2000x300,128x3000x200,256x1500x600,64x4000x150,256x300x2000,256x700x700 \
  timeout -k 10 300 python3 -u tools/fp64_split_batch.py $O/fp64_split_skinny.txt > $O/fp64_split_skinny.log 2>&1
echo finished
