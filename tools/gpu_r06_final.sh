#!/bin/bash
# Round-6 evidence: full GPU suite, smoke, the default bench line (PMC traffic + issue passes, both CPU legs), every
# other workload with its oracle sample, the unchanged callers (per-call latency, GUI call breakdown, process model,
# timing.py loop), fp64 per-call scan, script calls, c4 kernel traces (2 parts; 1 part = SED_CK_HALVES=1) and an SQ
# pass.  Outputs under gpurun_out/<dir>/, copied to profiles/r06/final/.
set -e
O=gpurun_out/${1:-r06final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_c4.json 2> $O/bench_c4.log
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print({k: d.get(k) for k in ('value','ms_per_step','script_valid_rate','script_exact_rate')})"
for w in c3 c2 c5 c5n iupac timing; do
  timeout -k 10 300 python3 bench.py --workload $w --traffic none --no-python-baseline --cpu-seconds 5 >> $O/bench_other.jsonl 2>> $O/bench_other.log
done
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
timeout -k 10 200 python3 tools/call_breakdown.py > $O/call_breakdown.txt 2>&1
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
timeout -k 10 300 python3 tools/timing_breakdown.py $O/timing_breakdown.txt > /dev/null 2>&1
timeout -k 10 200 python3 tools/fp64_call_scaling.py $O/fp64_call_scaling.txt > /dev/null 2>&1
timeout -k 10 200 python3 tools/script_calls.py > $O/script_calls.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $PWD/$O/kt_c4 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c4.json 2> $O/kt_c4.log
SED_CK_HALVES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $PWD/$O/kt_c4_1part -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c4_1part.json 2> $O/kt_c4_1part.log
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -T -d $PWD/$O/sq_c4 -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_c4.json 2> $O/sq_c4.log
echo finished
