#!/bin/bash
# Round-5 batch 15: M5 kernel stats of the graph-replayed step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b15; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 8
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 23 40 > $O/kstats_m5.txt 2>&1; cat $O/kstats_m5.txt
