#!/bin/bash
# Round 4: fp64 issue costs (tools/ubench/valu_f64.hip)
set -e
O=gpurun_out/${1:-r04s7}
mkdir -p $O
timeout -k 10 120 tools/ubench/valu_f64 > $O/ubench_valu_f64.txt 2>&1
cat $O/ubench_valu_f64.txt
