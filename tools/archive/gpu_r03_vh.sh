#!/bin/bash
# select-free hold fixed: the CK/route GPU tests on the VHOLD build, c4 A/B against the current build; fp64 R auto
set -e
O=gpurun_out/r03vh
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests_rccl.log 2>&1; tail -2 $O/tests_rccl.log
SED_LIBRARY=$PWD/tools/ab_libs/libsed_vhold.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_routes.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_vhold.log 2>&1
tail -2 $O/tests_vhold.log
tools/ab2.sh r03vh_ab 3 tools/ab_libs/libsed_cur.so tools/ab_libs/libsed_vhold.so
cat gpurun_out/r03vh_ab/ab.jsonl
for w in timing iupac; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --traffic none > $O/f.json 2>> $O/f.log
  python3 -c "import json; d=json.load(open('$O/f.json')); print(json.dumps({'w':'$w','R':d['config']['rows_per_lane'],'step_ms':d['ms_per_step'],'valid':d.get('script_valid_rate')}))" >> $O/fp64_auto.jsonl
done
cat $O/fp64_auto.jsonl
