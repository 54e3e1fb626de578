#!/bin/bash
# Round 6 step 3: the fp64 SPLIT gate tests, then the CK forward's LDS prefetch (SED_CK_TVPF=1 build) A/B on c4
set -e
O=gpurun_out/${1:-r06s3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "fp64_split" > $O/tests.log 2>&1
tail -2 $O/tests.log
bash tools/ab_env.sh ${1:-r06s3} 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_pf1.so"
cat $O/ab.jsonl
echo finished
