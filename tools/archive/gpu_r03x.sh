#!/bin/bash
# halves default: full GPU suite, default bench line (PMC passes), A/B off/on
set -e
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
timeout -k 10 400 python3 bench.py --no-python-baseline --cpu-seconds 5 > $O/bench_c4.json 2> $O/bench_c4.log
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print({k: d.get(k) for k in ('value','ms_per_step','script_valid_rate','script_exact_rate')}, d['roofline'], d.get('issue'))"
tools/ab_env.sh r03x_ab 2 "SED_CK_HALVES=1" "-" "SED_CK_HALVES=3" "SED_CK_HALVES=4"
cat gpurun_out/r03x_ab/ab.jsonl
