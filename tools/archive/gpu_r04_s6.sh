#!/bin/bash
# Round 4: the fp64 kernel's U-space path-length keys and LDS chunk rows (top row, symbols, bottom cells through LDS
# instead of DPP rotations): every GPU test, then iupac / timing interleaved against the previous build, and one SQ
# pass of iupac
set -e
O=gpurun_out/${1:-r04s6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
tail -3 $O/tests.log
AB_ARGS="--workload iupac" timeout -k 10 300 bash tools/ab2.sh ${1:-r04s6}/iupac 2 tools/ab_libs/libsed_prev.so rna-sequence-diff-patch_amd/libsed.so
cat $O/iupac/ab.jsonl
AB_ARGS="--workload timing" timeout -k 10 300 bash tools/ab2.sh ${1:-r04s6}/timing 2 tools/ab_libs/libsed_prev.so rna-sequence-diff-patch_amd/libsed.so
cat $O/timing/ab.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -T -d $O/sq_iupac -o sq --output-format csv -- python3 bench.py --workload iupac --steps 1 --warmup 0 --no-cpu-baseline --traffic none > $O/sq_iupac.json 2> $O/sq_iupac.log
echo finished
