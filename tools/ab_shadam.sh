#!/bin/bash
# SH Adam fused into the SH-colour backward: trainer GPU tests, M2 bench
# off / on x2, kernel stats with it on.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/shadam; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_fit.py tests/test_gpu_strategy.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    GSPLAT_HIP_SH_ADAM_IN_BWD=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_f$f.$r.json 2>/dev/null || exit 2
  done
done
GSPLAT_HIP_SH_ADAM_IN_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 3
exit 0
