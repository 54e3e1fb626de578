#!/bin/bash
# Round 6 step 21: the dot-key factorisation memoised per thread (dot_keys: ~75 us per call on the build host): the
# parity, route and module GPU tests, the GUI engine call timeline and the per-call latency
set -e
O=$PWD/gpurun_out/${1:-r06s21}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or parity or shim" > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 120 python3 tools/gui_engine_calls.py > $O/gui_engine_calls.txt 2>&1
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
timeout -k 10 200 python3 tools/call_breakdown.py > $O/call_breakdown.txt 2>&1
cat $O/gui_engine_calls.txt $O/call_latency.txt $O/call_breakdown.txt
echo finished
