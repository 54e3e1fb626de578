#!/bin/bash
# Round 4: c4 with uneven parts (SED_CK_PART0, since removed: part 0's share in per mille): 400, 450, 500 (default), 550, 600
set -e
O=gpurun_out/${1:-r04s10}
mkdir -p $O
export TMPDIR=/tmp
SED_CK_PART0=450 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_routes.py -m gpu -k "parts_on_streams or headline" > $O/tests_part0.log 2>&1
tail -2 $O/tests_part0.log
timeout -k 10 900 bash tools/ab_env.sh ${1:-r04s10}/ab 2 - SED_CK_PART0=400 SED_CK_PART0=450 SED_CK_PART0=550 SED_CK_PART0=600
cat $O/ab/ab.jsonl
