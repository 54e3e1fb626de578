#!/bin/bash
# select-free hold: per-tile dumps of both debug builds on the failing 208 x 106 pair; fp64 R A/B; parts timing
set -e
O=gpurun_out/r03dbg
mkdir -p $O
export TMPDIR=/tmp
for L in libsed_dbg0 libsed_dbg1; do
  SED_LIBRARY=$PWD/tools/ab_libs/$L.so timeout -k 10 120 python3 -u tools/diag_vhold_dump.py >> $O/dumps.jsonl 2>> $O/dumps.err
done
bash tools/gpu_r03z.sh
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --traffic none > $O/c4_parts_times.json 2> $O/c4.log
python3 -c "import json; d=json.load(open('$O/c4_parts_times.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['traceback_ms'], d['roofline']['frac'], d['roofline']['frac_step'])"
