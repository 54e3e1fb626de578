#!/bin/bash
# config 3 CHAIN kernel: kernel trace + SQ issue/stall counters (separate passes)
set -e
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_bench.json 2> $O/kt.log
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/sq -o sq -- python3 bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_bench.json 2> $O/sq.log
find $O -name "*.csv" | head -20
