#!/bin/bash
# Round 4: SPLIT checkpoint route for config 2 (SED_OPT_SPLITCK): its parity tests, then config 2 against the ladder-key
# route, 3 interleaved rounds, and a kernel trace of each
set -e
O=gpurun_out/${1:-r04s11}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -k "split or stripe_parallel or config2 or g3" > $O/tests.log 2>&1
tail -3 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --workload c2 --traffic none --no-cpu-baseline >> $O/ab_c2.jsonl 2>> $O/ab_c2.log
  timeout -k 10 200 python3 bench.py --workload c2 --traffic none --no-cpu-baseline --no-split-ck >> $O/ab_c2.jsonl 2>> $O/ab_c2.log
done
python3 -c "
import json
for l in open('$O/ab_c2.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config']['traceback'], round(d['ms_per_step'],4), d['roofline'].get('kernel_ms_per_step'), d.get('traceback_ms'), d.get('script_valid_rate'), d.get('script_exact_rate'))
"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c2 -o kt --output-format csv -- python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --traffic none > $O/kt_c2.json 2> $O/kt_c2.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c2_old -o kt --output-format csv -- python3 bench.py --workload c2 --steps 20 --warmup 2 --no-cpu-baseline --traffic none --no-split-ck > $O/kt_c2_old.json 2> $O/kt_c2_old.log
head -6 $O/kt_c2/kt_kernel_stats.csv $O/kt_c2_old/kt_kernel_stats.csv
