#!/bin/bash
# Step-level GPU idle: rocprofv3 kernel trace of the M2 bench (gaps between
# kernels per step), the host timeline of one step, and three plain benches.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${GR_TAG:-gaps}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 1
python tools/step_timeline.py $O/trace/run_kernel_trace.csv > $O/timeline.txt || exit 2
timeout -k 10 300 python -u tools/host_timeline.py > $O/host_timeline.txt 2>&1 || exit 3
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench$i.json 2>/dev/null || exit 4
done
exit 0
