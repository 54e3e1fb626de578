#!/bin/bash
# c4 checkpoint path: CK GPU tests, bench line, kernel trace and two SQ counter passes -> gpurun_out/$TAG/
set -e
TAG=${1:-pmc}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or g3 or ladder" > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_bench.json 2> $O/kt_bench.log
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -T -d $O/sq1 -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq1.json 2> $O/sq1.log
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_VMEM -T -d $O/sq2 -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq2.json 2> $O/sq2.log
