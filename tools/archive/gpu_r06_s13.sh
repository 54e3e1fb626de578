#!/bin/bash
# Round 6 step 13: two-chunk windows at 5 waves per SIMD (the new default): the route, parity and fuzz tests, then c4
# A/B against the entry word's LDS reads hoisted (eh1), 6 waves per SIMD (w6) and the round's previous build (head)
set -e
O=$PWD/gpurun_out/${1:-r06s13}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or fuzz or parity" > $O/tests.log 2>&1
tail -2 $O/tests.log
AB_ARGS="" bash tools/ab_env.sh ${1:-r06s13}/c4 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_eh1.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_w6.so" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_head.so"
cat $O/c4/ab.jsonl
echo finished
