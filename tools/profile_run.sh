#!/bin/bash
# Kernel-trace stats of the bench workload (per-kernel average durations; the
# rasterize_fwd row must agree with bench.py's roofline.launch_ms), then the
# default bench line (roofline.traffic from its own PMC child runs, and the
# CPU baseline).  Usage (on the GPU box): bash tools/profile_run.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 2
exit 0
