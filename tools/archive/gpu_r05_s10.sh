#!/bin/bash
# Round 5, step 10: unchanged-caller paths after the batched host fast paths (forked per-document loop and forked
# wfsearch), config-3 checkpoint A/B, fp64 timing A/B (rows per lane, segments) with an SQ pass
set -e
O=gpurun_out/${1:-r05s10}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
cat $O/caller_paths.txt
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --traffic none"
for r in 1 2; do
  for a in "" "--tb 2" ; do
    timeout -k 10 200 $B --workload c3 $a > $O/c3.json 2>> $O/c3.log
    python3 -c "import json; d=json.load(open('$O/c3.json')); print(json.dumps({'args':'$a','round':$r,'value':d['value'],'step_ms':d['ms_per_step'],'exact':d.get('script_exact_rate'),'tb_ms':d.get('traceback_ms'),'dp_ms':d['roofline'].get('kernel_ms')}))" >> $O/c3_ab.jsonl
  done
  for a in "" "--rows-per-lane 8" "--seg 2"; do
    timeout -k 10 200 $B --workload timing $a > $O/timing.json 2>> $O/timing.log
    python3 -c "import json; d=json.load(open('$O/timing.json')); print(json.dumps({'args':'$a','round':$r,'value':d['value'],'step_ms':d['ms_per_step'],'exact':d.get('script_exact_rate'),'dp_ms':d['roofline'].get('kernel_ms')}))" >> $O/timing_ab.jsonl
  done
done
cat $O/c3_ab.jsonl $O/timing_ab.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/pmc_timing -o pmc --output-format csv -- python3 bench.py --workload timing --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/pmc_timing.log 2>&1
python3 - <<PY
import csv, glob
for f in glob.glob('$O/pmc_timing/**/*counter_collection.csv', recursive=True):
    agg = {}
    for r in csv.DictReader(open(f)):
        agg.setdefault(r['Kernel_Name'][:50], {}).setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    for k, c in agg.items():
        print(k, {n: '%.3g' % (sum(x) / len(x)) for n, x in c.items()}, 'launches', len(next(iter(c.values()))))
PY
