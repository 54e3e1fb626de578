#!/bin/bash
# Round 4: c4 schedule A/B (SED_CK_SCHED=1, since removed: forwards back to back on one stream vs the default staggered parts) with
# the parts timeline, and the fp64 segment cost model's picks (timing, iupac, timing at R = 8)
set -e
O=gpurun_out/${1:-r04s5}
mkdir -p $O
export TMPDIR=/tmp
# the traceback's scalar-base loads first: every checkpoint route (R = 4, 8, 16; stripe and chain; dot keys; parts;
# the headline route)
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_routes.py -m gpu -k "checkpoint or headline or dot_keys" > $O/tests_ck.log 2>&1
tail -3 $O/tests_ck.log
# CK chunk loop: 2 (default), 4 or 8 groups per iteration, interleaved
timeout -k 10 400 bash tools/ab2.sh ${1:-r04s5}/unroll 2 rna-sequence-diff-patch_amd/libsed.so tools/ab_libs/libsed_u4.so tools/ab_libs/libsed_u8.so
cat $O/unroll/ab.jsonl
timeout -k 10 200 python3 tools/c4_timeline.py 20 > $O/timeline_default.txt 2>&1
SED_CK_SCHED=1 timeout -k 10 200 python3 tools/c4_timeline.py 20 > $O/timeline_sched.txt 2>&1
cat $O/timeline_default.txt $O/timeline_sched.txt
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --traffic none --no-cpu-baseline >> $O/ab_sched.jsonl 2>> $O/ab_sched.log
  SED_CK_SCHED=1 timeout -k 10 300 python3 bench.py --traffic none --no-cpu-baseline >> $O/ab_sched.jsonl 2>> $O/ab_sched.log
done
for w in timing iupac; do
  timeout -k 10 300 python3 bench.py --workload $w --traffic none --no-cpu-baseline >> $O/fp64_auto.jsonl 2>> $O/fp64_auto.log
done
timeout -k 10 300 python3 bench.py --workload timing --rows-per-lane 8 --traffic none --no-cpu-baseline >> $O/fp64_auto.jsonl 2>> $O/fp64_auto.log
echo finished
