#!/bin/bash
# Round 4, last check of the final code: every GPU test, smoke, the default bench line, config 2
set -e
O=gpurun_out/${1:-r04check}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench_c4.json 2> $O/bench_c4.log
timeout -k 10 300 python3 bench.py --workload c2 --traffic none --no-python-baseline --cpu-seconds 5 > $O/bench_c2.json 2> $O/bench_c2.log
python3 -c "
import json
for f in ('$O/bench_c4.json', '$O/bench_c2.json'):
    d = json.loads(open(f).read().strip().split(chr(10))[-1])
    print(d['config']['workload'][:20], d['ms_per_step'], d['value'], d.get('script_valid_rate'), d.get('script_exact_rate'))
"
