#!/bin/bash
# cells/s of the c4 shape at pair counts around the resident-wave rounds (5120 waves = 1024 SIMDs x 5)
set -e
O=gpurun_out/${1:-tail}
mkdir -p $O
export TMPDIR=/tmp
for p in 5120 8192 10240 2560; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --pairs $p --steps 10 >> $O/tail.jsonl 2>> $O/log
done
