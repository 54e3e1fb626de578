#!/bin/bash
# Round 6 step 4: the banded emit walk (one wave per 64-row band; SED_TB_BANDEMIT) -- the stripe-parallel and SPLIT
# route tests, the route fuzz, then the script calls interleaved against the per-stripe emit (libsed_be0.so) and a
# kernel trace of the calls
set -e
O=gpurun_out/${1:-r06s4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "stripe or split or fuzz or shim or g3 or config2" > $O/tests.log 2>&1
tail -2 $O/tests.log
for r in 1 2 3; do
  echo "round $r default" >> $O/script_calls.txt
  timeout -k 10 120 python3 tools/script_calls.py >> $O/script_calls.txt 2>&1
  echo "round $r be0" >> $O/script_calls.txt
  SED_LIBRARY=$PWD/tools/ab_libs/libsed_be0.so timeout -k 10 120 python3 tools/script_calls.py >> $O/script_calls.txt 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 tools/script_calls.py > $O/kt.log 2>&1
cat $O/script_calls.txt
echo finished
