#!/bin/bash
# Round 6 step 17: generate_es lists released by the caller are reused as the next script call's records
# (es_recycle): the module and host GPU tests, then the GUI call latency and its breakdown
set -e
O=gpurun_out/${1:-r06s17}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_shim_gpu.py tests/test_fuzz_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
timeout -k 10 200 python3 tools/call_breakdown.py > $O/call_breakdown.txt 2>&1
cat $O/call_latency.txt $O/call_breakdown.txt
echo finished
