#!/bin/bash
# Round 5, step 1: the new route tests (SPLIT window walk, empty-side SPLIT batch, two residency rounds of the
# checkpoint route), the whole routes file, smoke, the default bench line with its strided oracle sample
set -e
O=gpurun_out/${1:-r05s1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_routes.log 2>&1
tail -2 $O/tests_routes.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench_c4.json 2> $O/bench_c4.log
python3 -c "
import json
d = json.loads(open('$O/bench_c4.json').read().strip().split(chr(10))[-1])
print(d['ms_per_step'], d['value'], d.get('script_valid_rate'), d.get('script_exact_rate'), d.get('exact_sample'))
"
