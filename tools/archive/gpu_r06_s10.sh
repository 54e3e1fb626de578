#!/bin/bash
# Round 6 step 10: where config 3's padding-zeroing cost goes -- per-kernel durations (rocprofv3 --kernel-trace
# --stats) of the c3 bench for the default build (zeroing after the walk), SED_PAD_EARLY=1 (zeroing before the walk)
# and SED_PAD_ZERO=0 (none), then an interleaved A/B of the three
set -e
O=$PWD/gpurun_out/${1:-r06s10}
mkdir -p $O
export TMPDIR=/tmp
for v in def pe1 pz0; do
  if [ $v = def ]; then EV=""; else EV="SED_LIBRARY=$PWD/tools/ab_libs/libsed_$v.so"; fi
  env $EV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run -- python3 bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --traffic none > $O/bench_$v.json 2> $O/bench_$v.log
  f=$(find $O/kt_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -i traceback $f || true
done
AB_ARGS="--workload c3" bash tools/ab_env.sh ${1:-r06s10}/c3 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pe1.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pz0.so"
cat $O/c3/ab.jsonl
echo finished
