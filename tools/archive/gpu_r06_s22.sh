#!/bin/bash
# Round 6 step 22: band-map walks capped at 96 + 64 ceil(m / n) steps (SED_TBMAP_CAP): the route, parity, module and
# fuzz GPU tests, the script calls' kernel times with and without the cap, c2 A/B and the GUI call latency
set -e
O=$PWD/gpurun_out/${1:-r06s22}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "routes or parity or shim or fuzz" > $O/tests.log 2>&1
tail -2 $O/tests.log
for v in def cap0; do
  if [ $v = def ]; then EV=""; else EV="SED_LIBRARY=$PWD/tools/ab_libs/libsed_$v.so"; fi
  env $EV timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python3 tools/script_calls.py > $O/script_calls_$v.txt 2> $O/script_calls_$v.log
  cat $O/script_calls_$v.txt
done
AB_ARGS="--workload c2" bash tools/ab_env.sh ${1:-r06s22}/c2 3 "-" "SED_LIBRARY=$PWD/tools/ab_libs/libsed_cap0.so"
timeout -k 10 200 python3 tools/call_latency.py > $O/call_latency.txt 2>&1
cat $O/c2/ab.jsonl $O/call_latency.txt
echo finished
