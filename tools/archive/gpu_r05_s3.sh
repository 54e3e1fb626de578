#!/bin/bash
# Round 5, step 3: the forward-lane replay traceback (sed_traceback_ckr_kernel): route/parity tests at the default
# (replay at R = 16), the checkpoint tests with the replay at every R, then c4 A/B against the lane-per-row sweep
set -e
O=gpurun_out/${1:-r05s3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
SED_CK_REPLAY=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py -m gpu -x -v -k "checkpoint or chain or ck or headline" --timeout 300 --timeout-method thread > $O/tests_replay_all.log 2>&1
tail -1 $O/tests_replay_all.log
for r in 1 2; do
  for v in 1 0; do
    SED_CK_REPLAY=$v timeout -k 10 300 python3 bench.py --traffic none --no-python-baseline --cpu-seconds 3 >> $O/ab.jsonl 2>> $O/ab.log
  done
done
python3 -c "
import json
for l in open('$O/ab.jsonl'):
    d = json.loads(l)
    print(d['config']['env'], round(d['ms_per_step'], 3), round(d['roofline']['kernel_ms_per_step'], 3), round(d['traceback_ms'], 3), d.get('script_exact_rate'), d.get('script_valid_rate'))
"
