#!/bin/bash
# Round 5, step 20: the checkpoint traceback's word loop with `continue` instead of `break` at R = 16
# (SED_CK_SWEEP_CONT build): c4 A/B and the traceback's SQ counters in one part
set -e
O=gpurun_out/${1:-r05s20}
mkdir -p $O
export TMPDIR=/tmp
CT=SED_LIBRARY=$PWD/tools/ab_libs/libsed_cont.so
bash tools/ab_env.sh ${1:-r05s20} 3 "-" "$CT"
cat $O/ab.jsonl
for v in def cont; do
  if [ $v = cont ]; then E="$CT"; else E=""; fi
  env $E SED_CK_HALVES=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -T -d $O/pmc_$v -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/pmc_$v.log 2>&1
done
python3 - <<PY
import csv, glob
for v in ('def', 'cont'):
    for f in glob.glob('$O/pmc_%s/**/*counter_collection.csv' % v, recursive=True):
        agg = {}
        for r in csv.DictReader(open(f)):
            if 'traceback' in r['Kernel_Name']:
                agg.setdefault(r['Kernel_Name'][:30], {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        for k, c in agg.items():
            print(v, k, {n: '%.3g' % (sum(x) / len(x)) for n, x in c.items()})
PY
