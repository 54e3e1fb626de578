#!/bin/bash
# Round 6 step 20: host API and kernel timeline of the GUI call's engine part (tools/gui_engine_calls.py)
set -e
O=$PWD/gpurun_out/${1:-r06s20}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/gui_engine_calls.py > $O/plain.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/rt -o rt --output-format csv -- python3 tools/gui_engine_calls.py > $O/traced.txt 2> $O/traced.log
cat $O/plain.txt
ls $O/rt
echo finished
