#!/bin/bash
# part count and event placement, same box, 3 interleaved rounds
set -e
export TMPDIR=/tmp
tools/ab_env.sh r03y 3 "SED_CK_HALVES=1" "SED_CK_HALVES=2" "SED_CK_HALVES=2 SED_CK_PART_EVENTS=1" "SED_CK_HALVES=3" "SED_CK_HALVES=3 SED_CK_PART_EVENTS=1"
cat gpurun_out/r03y/ab.jsonl
