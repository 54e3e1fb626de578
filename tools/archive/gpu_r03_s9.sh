#!/bin/bash
# round 3, session 2: CK forward at 4 vs 5 waves per SIMD with 2 parts (c4, 3 interleaved rounds)
set -e
tools/ab2.sh r03s9_waves 3 tools/ab_libs/libsed_cur.so tools/ab_libs/libsed_w4.so
cat gpurun_out/r03s9_waves/ab.jsonl
