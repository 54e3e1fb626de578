#!/bin/bash
# Round 6 step 6: the GPU suite with the submit / wait pair API and the ES skeletons, then the GUI call's latency and
# breakdown, the host record build on the box's CPU, and a kernel trace of the script calls
set -e
O=gpurun_out/${1:-r06s6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
timeout -k 10 200 python3 tools/call_breakdown.py > $O/call_breakdown.txt 2>&1
timeout -k 10 200 python3 tools/es_build_bench.py > $O/es_build_bench.txt 2>&1
timeout -k 10 120 python3 tools/script_calls.py > $O/script_calls.txt 2>&1
cat $O/call_latency.txt $O/call_breakdown.txt $O/es_build_bench.txt $O/script_calls.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/kt -o kt --output-format csv -- python3 tools/script_calls.py > $O/kt.log 2>&1
find $O -name "*.csv" | head
echo finished
