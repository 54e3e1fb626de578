#!/bin/bash
# Round 4, first GPU call: the full GPU suite (with the headline-route test), the default bench line (spans-based
# roofline, PMC passes), and c4 kernel traces with 2 parts (default) and 1 part (SED_CK_HALVES=1: launches alone)
set -e
O=gpurun_out/${1:-r04s1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 600 python3 bench.py --no-python-baseline > $O/bench_c4.json 2> $O/bench_c4.log
cat $O/bench_c4.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c4 -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c4.json 2> $O/kt_c4.log
SED_CK_HALVES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_c4_1part -o kt --output-format csv -- python3 bench.py --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_c4_1part.json 2> $O/kt_c4_1part.log
for w in c5n c5; do
  timeout -k 10 300 python3 bench.py --workload $w --traffic none --no-python-baseline --cpu-seconds 3 >> $O/bench_c5.jsonl 2>> $O/bench_c5.log
done
timeout -k 10 300 python3 bench.py --workload c5n --no-scaled --traffic none --no-python-baseline --cpu-seconds 3 >> $O/bench_c5.jsonl 2>> $O/bench_c5.log
timeout -k 10 300 python3 bench.py --workload c5n --traffic none --no-python-baseline --cpu-seconds 3 >> $O/bench_c5.jsonl 2>> $O/bench_c5.log
timeout -k 10 120 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
echo finished
