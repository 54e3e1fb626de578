#!/bin/bash
# Round 4: fp64 kernel occupancy (SED_F64_WAVES 4 / 5, a knob since removed, against the free allocation), iupac and timing, 2 rounds
set -e
O=gpurun_out/${1:-r04s12}
mkdir -p $O
export TMPDIR=/tmp
AB_ARGS="--workload iupac" timeout -k 10 400 bash tools/ab2.sh ${1:-r04s12}/iupac 2 rna-sequence-diff-patch_amd/libsed.so tools/ab_libs/libsed_fw4.so tools/ab_libs/libsed_fw5.so
cat $O/iupac/ab.jsonl
AB_ARGS="--workload timing" timeout -k 10 400 bash tools/ab2.sh ${1:-r04s12}/timing 2 rna-sequence-diff-patch_amd/libsed.so tools/ab_libs/libsed_fw4.so tools/ab_libs/libsed_fw5.so
cat $O/timing/ab.jsonl
