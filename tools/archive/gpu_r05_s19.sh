#!/bin/bash
# Round 5, step 19: where a forked child's batched search spends its time (cProfile of a repeated search in the child)
set -e
O=gpurun_out/${1:-r05s19}
mkdir -p $O
export TMPDIR=/tmp
CALLER_PATHS_PROFILE=$PWD/$O/child_profile.txt timeout -k 10 300 python3 tools/caller_paths.py $O/caller_paths.json > $O/caller_paths.txt 2>&1
cat $O/caller_paths.txt
head -60 $O/child_profile.txt
