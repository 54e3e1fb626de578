#!/bin/bash
# Round 6 step 5: the forward step's chain microbenchmark (one 17-deep chain vs two 8-deep chains per step, 1-6 waves
# per SIMD), and where the drop-in GUI call's time goes (engine vs host, tools/call_breakdown.py, call_latency.py)
set -e
O=gpurun_out/${1:-r06s5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench/dot_chain > $O/dot_chain.txt 2>&1
cat $O/dot_chain.txt
timeout -k 10 200 python3 tools/call_breakdown.py > $O/call_breakdown.txt 2>&1
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
cat $O/call_breakdown.txt $O/call_latency.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/script_calls.py > $O/kt.log 2>&1
ls -la $O/kt
cp $O/kt/*.csv $O/ 2>/dev/null || true
echo finished
