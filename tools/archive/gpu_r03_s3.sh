#!/bin/bash
# round 3, session 2: every GPU test on the current build (bit-parallel lane kernels, fp64 plain-chunk loop, select-free
# hold on), the fp64 A/B (previous build vs the plain-chunk loop) on iupac and timing, c5n with / without bit-parallel
set -e
O=gpurun_out/r03s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
for r in 1 2; do
  for f in "" "--no-bitpar"; do
    timeout -k 10 120 python3 bench.py --workload c5n --steps 200 --warmup 5 --no-cpu-baseline --traffic none $f > $O/c5n.json 2>> $O/c5n.log
    python3 -c "import json; d=json.load(open('$O/c5n.json')); print(json.dumps({'flag':'$f','value':d['value'],'step_ms':d['ms_per_step'],'dp_ms':d['roofline']['kernel_ms'],'bitpar':d['config'].get('bitpar_pairs'),'exact':d.get('dist_exact_rate')}))" >> $O/c5n_ab.jsonl
  done
done
cat $O/c5n_ab.jsonl
for w in iupac timing; do
  AB_ARGS="--workload $w" tools/ab2.sh r03s3_f64_$w 2 tools/ab_libs/libsed_cur.so tools/ab_libs/libsed_f64plain.so
  cat gpurun_out/r03s3_f64_$w/ab.jsonl
done
