#!/bin/bash
# round 3, session 2: RCCL gather test, bit-parallel lane kernel tests + c5 A/B, select-free hold tests + c4 A/B
set -e
O=gpurun_out/r03s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_dist_gpu.py "tests/test_gpu_parity.py::test_lane_bitpar_unit_costs_vs_oracle" "tests/test_gpu_parity.py::test_lane_bitpar_needs_unit_costs" "tests/test_gpu_parity.py::test_lane_x2_packed_distance_vs_oracle" "tests/test_gpu_parity.py::test_lane_kernel_all_vs_all_shape" "tests/test_gpu_parity.py::test_lane_kernel_short_str2_vs_oracle" -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests_new.log 2>&1
tail -3 $O/tests_new.log
for r in 1 2 3; do
  for f in "" "--no-bitpar"; do
    timeout -k 10 120 python3 bench.py --workload c5 --steps 200 --warmup 5 --no-cpu-baseline --traffic none $f > $O/c5.json 2>> $O/c5.log
    python3 -c "import json; d=json.load(open('$O/c5.json')); print(json.dumps({'flag':'$f','value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'kernel':d['roofline']['kernel'],'exact':d.get('dist_exact_rate')}))" >> $O/c5_ab.jsonl
  done
done
cat $O/c5_ab.jsonl
SED_LIBRARY=$PWD/tools/ab_libs/libsed_vhold.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_routes.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or ck or route" > $O/tests_vhold.log 2>&1
tail -3 $O/tests_vhold.log
tools/ab2.sh r03s2_vh 3 tools/ab_libs/libsed_cur.so tools/ab_libs/libsed_vhold.so
cat gpurun_out/r03s2_vh/ab.jsonl
