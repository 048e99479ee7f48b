#!/bin/bash
# Kernel-trace stats of the bench workload + HBM traffic passes for the
# rasterizer kernels.  Usage (on the GPU box): bash tools/profile_run.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit 1
R='r16'
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE -f csv -d $OUT/fetch -o p -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc WRITE_SIZE -f csv -d $OUT/write -o p -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1 || exit 3
exit 0
