#!/bin/bash
# A/B: checkpoint batches sequential (default) vs pipelined (traceback k beside DP k+1), interleaved rounds
set -e
O=gpurun_out/${1:-abpipe}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 >> $O/seq.jsonl 2>> $O/log
  SED_CK_PIPELINE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 >> $O/pipe.jsonl 2>> $O/log
done
