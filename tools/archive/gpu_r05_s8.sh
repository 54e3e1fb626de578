#!/bin/bash
# Round 5, step 8: the quarter-band traceback with the asm scalar walk: tests, A/B (1 and 2 parts), SQ counters
set -e
O=gpurun_out/${1:-r05s8}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
bash tools/ab_env.sh ${1:-r05s8} 2 "SED_CK_REPLAY=0" "-" "SED_CK_REPLAY=0 SED_CK_HALVES=1" "SED_CK_HALVES=1"
cat $O/ab.jsonl
for v in 2 0; do
  SED_CK_REPLAY=$v SED_CK_HALVES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/pmc_$v -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/pmc_$v.log 2>&1
done
python3 - <<PY
import csv, glob
for v in (2, 0):
    for f in glob.glob('$O/pmc_%d/**/*counter_collection.csv' % v, recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if 'traceback' in r['Kernel_Name']:
                agg.setdefault(r['Kernel_Name'][:40], {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        for k, c in agg.items():
            print(v, k, {n: '%.3g' % (sum(x) / len(x)) for n, x in c.items()})
PY
