#!/bin/bash
# Round 6 step 7: config 4 at R = 16 (default) and R = 8 (9-deep chains, twice the DPP moves and ramp) with the SQ
# issue pass, and config 4 in one part (kernel trace) for the forward alone
set -e
O=gpurun_out/${1:-r06s7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c4_r16.json 2> $O/c4_r16.log
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --rows-per-lane 8 > $O/c4_r8.json 2> $O/c4_r8.log
python3 -c "
import json
for f in ('c4_r16','c4_r8'):
    d = json.load(open('$O/%s.json' % f))
    print(f, 'step', round(d['ms_per_step'],3), 'dp', round(d['roofline']['kernel_ms_mean_launch'],3), 'tb', round(d['traceback_ms'],3), 'issue', json.dumps(d.get('issue')), 'valid', d.get('script_valid_rate'))"
echo finished
