#!/bin/bash
# Round 6 check: GPU parity suite (or a -k selection), then the c4 / c3 / c2 bench lines without CPU legs
set -e
O=gpurun_out/${1:-r06chk}
SEL=${2:-}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$SEL" > $O/tests.log 2>&1
else
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
fi
tail -2 $O/tests.log
for w in c4 c3 c2; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 2 --no-cpu-baseline --traffic none >> $O/bench.jsonl 2>> $O/bench.log
done
python3 -c "
import json
for l in open('$O/bench.jsonl'):
    d = json.loads(l); print(d['config'].get('workload'), d['ms_per_step'], d.get('script_exact_rate'))"
echo finished
