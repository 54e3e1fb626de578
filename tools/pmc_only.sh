#!/bin/bash
# Two SQ counter passes over one c4 bench step -> gpurun_out/$TAG/sq{1,2}
set -e
TAG=${1:-pmc}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -T -d $O/sq1 -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} --traffic none > $O/sq1.json 2> $O/sq1.log
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VMEM -T -d $O/sq2 -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} --traffic none > $O/sq2.json 2> $O/sq2.log
