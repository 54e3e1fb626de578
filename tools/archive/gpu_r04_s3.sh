#!/bin/bash
# Round 4, third GPU call: the fp64 route's evidence (item 4 of VERDICT r03): iupac and timing bench lines, kernel
# traces, and SQ passes (VALU / SALU / LDS / wait / wave cycles) of one step each; plus the c4 traceback's SQ wait pass
set -e
O=gpurun_out/${1:-r04s3}
mkdir -p $O
export TMPDIR=/tmp
for w in iupac timing; do
  timeout -k 10 300 python3 bench.py --workload $w --traffic none --no-python-baseline --cpu-seconds 3 > $O/bench_$w.json 2> $O/bench_$w.log
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $O/kt_$w -o kt --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 1 --no-cpu-baseline --traffic none > $O/kt_$w.json 2> $O/kt_$w.log
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/sq_$w -o sq --output-format csv -- python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_$w.json 2> $O/sq_$w.log
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/sq_c4 -o sq --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_c4.json 2> $O/sq_c4.log
for R in 4 8; do
  timeout -k 10 300 python3 bench.py --workload timing --rows-per-lane $R --traffic none --no-cpu-baseline >> $O/bench_timing_R.jsonl 2>> $O/bench_timing_R.log
done
echo finished
