#!/bin/bash
# round 3, session 2: fp64 rows per lane 16 (A/B against 8 / 4 on iupac and timing), checkpoint parts 2/3/4 on c4
set -e
O=gpurun_out/r03s7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "iupac or fp64 or g2 or edge" > $O/tests_f64.log 2>&1
tail -2 $O/tests_f64.log
for r in 1 2; do
  for a in "--workload iupac --rows-per-lane 8" "--workload iupac --rows-per-lane 16" "--workload timing --rows-per-lane 4" "--workload timing --rows-per-lane 16"; do
    timeout -k 10 200 python3 bench.py $a --steps 10 --warmup 2 --no-cpu-baseline --traffic none > $O/x.json 2>> $O/x.log
    python3 -c "import json; d=json.load(open('$O/x.json')); print(json.dumps({'args':'$a','value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'tb_ms':d.get('traceback_ms'),'valid':d.get('script_valid_rate'),'exact':d.get('script_exact_rate')}))" >> $O/f64_R.jsonl
  done
done
cat $O/f64_R.jsonl
tools/ab_env.sh r03s7_parts 2 "SED_CK_HALVES=2" "-" "SED_CK_HALVES=4"
cat gpurun_out/r03s7_parts/ab.jsonl
