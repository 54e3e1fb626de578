#!/bin/bash
# Round 6 step 23: band-map walk cap base 64 (c64) and 256 staged columns (l256) against the default (cap base 96, 512
# columns): the script calls' kernel times per build, then the route / module / fuzz GPU tests on c64l256
set -e
O=$PWD/gpurun_out/${1:-r06s23}
mkdir -p $O
export TMPDIR=/tmp
for v in def c64 l256 c64l256; do
  if [ $v = def ]; then EV=""; else EV="SED_LIBRARY=$PWD/tools/ab_libs/libsed_$v.so"; fi
  env $EV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 tools/script_calls.py > $O/script_calls_$v.txt 2> $O/script_calls_$v.log
  echo "== $v"; cat $O/script_calls_$v.txt
done
SED_LIBRARY=$PWD/tools/ab_libs/libsed_c64l256.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or shim or fuzz" > $O/tests_c64l256.log 2>&1
tail -2 $O/tests_c64l256.log
echo finished
