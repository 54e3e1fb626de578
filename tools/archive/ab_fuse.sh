#!/bin/bash
# Fused checkpoint traceback (SED_CK_FUSE=1): CK tests under it, then an interleaved c4 A/B against the
# separate traceback kernel -> gpurun_out/$TAG/
set -e
O=gpurun_out/${1:-abfuse}
mkdir -p $O
export TMPDIR=/tmp
SED_CK_FUSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_routes.py tests/test_gpu_parity.py tests/test_shim_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "checkpoint or g3 or g8 or route or chain or corrupt or repeated" > $O/tests.log 2>&1
for r in 1 2; do
  SED_CK_FUSE=0 timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic none >> $O/sep.jsonl 2>> $O/log
  SED_CK_FUSE=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --traffic none >> $O/fused.jsonl 2>> $O/log
done
