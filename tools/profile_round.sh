#!/bin/bash
# Round profiling on the GPU box: bench line, rocprofv3 kernel-trace stats and
# the HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes, as
# MI355X_MICROARCH.md prescribes).  Usage: tools/profile_round.sh TAG
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_bench.json 2> $O/kt_bench.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline --traffic none > $O/fetch_bench.json 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/write -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline --traffic none > $O/write_bench.json 2>&1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -T -d $O/sq -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pipeline --traffic none > $O/sq_bench.json 2>&1
# secondary workloads: kernel-trace stats only (lane kernels for config 5, wave kernel at 512^2 for config 3)
for W in c3 c5 c5n; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/kt_$W -o kt --output-format csv -- python3 bench.py --workload $W --steps 20 --warmup 2 --no-cpu-baseline --traffic none > $O/kt_bench_$W.json 2> $O/kt_bench_$W.log
done
