#!/bin/bash
# Round 6 step 19: kernel timeline of the GUI's 4096^2 script call (tools/script_calls.py) to see the gaps between
# its kernels
set -e
O=$PWD/gpurun_out/${1:-r06s19}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 tools/script_calls.py > $O/script_calls.txt 2> $O/script_calls.log
ls -R $O | head
echo finished
