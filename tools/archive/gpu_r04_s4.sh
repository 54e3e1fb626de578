#!/bin/bash
# Round 4: fp64 16-lane segments — smoke (row-DPP self-test), the fp64 GPU tests, then timing / iupac A/B of
# SED_OPT_SEG auto vs 2 (never), interleaved
set -e
O=gpurun_out/${1:-r04s4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "segments or fp64 or iupac or g8 or f64" > $O/tests_f64.log 2>&1
tail -2 $O/tests_f64.log
for r in 1 2; do
  for w in timing iupac; do
    for sg in 0 2; do
      timeout -k 10 300 python3 bench.py --workload $w --seg $sg --traffic none --no-cpu-baseline >> $O/ab_seg.jsonl 2>> $O/ab_seg.log
    done
  done
done
timeout -k 10 300 python3 bench.py --workload timing --traffic none --no-python-baseline --cpu-seconds 3 > $O/bench_timing.json 2> $O/bench_timing.log
timeout -k 10 300 python3 bench.py --workload iupac --traffic none --no-python-baseline --cpu-seconds 3 > $O/bench_iupac.json 2> $O/bench_iupac.log
echo finished
