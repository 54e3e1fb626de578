#!/bin/bash
# round 3, session 2: two result slots aligned with the two streams for distance-only lane batches (libsed_2slot.so)
# against the current build: pipelined lane tests, c5 / c5n A/B, host enqueue overhead
set -e
O=gpurun_out/r03s11
mkdir -p $O
export TMPDIR=/tmp
SED_LIBRARY=$PWD/tools/ab_libs/libsed_2slot.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "pipelined or lane or bitpar" > $O/tests_2slot.log 2>&1
tail -2 $O/tests_2slot.log
for w in c5 c5n; do
  AB_ARGS="--workload $w --steps 200 --warmup 5" tools/ab2.sh r03s11_$w 3 tools/ab_libs/libsed_cur.so tools/ab_libs/libsed_2slot.so
  cat gpurun_out/r03s11_$w/ab.jsonl
done
timeout -k 10 200 python3 tools/host_overhead.py > $O/host_cur.txt 2>&1
SED_LIBRARY=$PWD/tools/ab_libs/libsed_2slot.so timeout -k 10 200 python3 tools/host_overhead.py > $O/host_2slot.txt 2>&1
cat $O/host_cur.txt $O/host_2slot.txt
