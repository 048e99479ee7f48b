#!/bin/bash
# Deferred SH Adam (side stream, bounded grid): trainer GPU tests, M2 bench
# with the update deferred off / on at several grid bounds, kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/defer2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fit.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  GSPLAT_HIP_DEFER_SH=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_off.$r.json 2>/dev/null || exit 2
  for b in 256 512 1024; do
    GSPLAT_HIP_DEFER_BLOCKS=$b timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_b$b.$r.json 2>/dev/null || exit 3
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 4
exit 0
