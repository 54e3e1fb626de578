#!/bin/bash
# Round 5, step 7: SQ counters of the quarter-band traceback and the lane-per-row sweep, one part (no overlap), one step
set -e
O=gpurun_out/${1:-r05s7}
mkdir -p $O
export TMPDIR=/tmp
for v in 2 0; do
  SED_CK_REPLAY=$v SED_CK_HALVES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/pmc_$v -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/pmc_$v.log 2>&1
done
python3 - <<PY
import csv, glob
for v in (2, 0):
    for f in glob.glob('$O/pmc_%d/**/*counter_collection.csv' % v, recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if 'traceback' in r['Kernel_Name'] or 'sed_wf' in r['Kernel_Name']:
                agg.setdefault(r['Kernel_Name'][:40], {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        for k, c in agg.items():
            print(v, k, {n: '%.3g' % (sum(x) / len(x)) for n, x in c.items()})
PY
