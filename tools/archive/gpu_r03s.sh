#!/bin/bash
# sel4 (no scratch copy of the cost tables) + SPLIT feeder: full GPU tests, then c3 / c4 / c2 A/B
set -e
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
AB_ARGS="--workload c3" tools/ab2.sh r03s_c3 3 tools/ab_libs/libsed_spb.so tools/ab_libs/libsed_sel4.so
tools/ab2.sh r03s_c4 2 tools/ab_libs/libsed_spb.so tools/ab_libs/libsed_sel4.so
AB_ARGS="--workload c2 --steps 200 --warmup 10" tools/ab2.sh r03s_c2 2 tools/ab_libs/libsed_spb.so tools/ab_libs/libsed_sel4.so
tail -3 $O/tests.log
cat gpurun_out/r03s_*/ab.jsonl
