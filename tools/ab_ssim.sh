#!/bin/bash
# Fused one-pass SSIM loss: trainer GPU tests, M2 bench with fused off / on,
# and kernel stats of the fused M2 step.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${AB_TAG:-ssimf}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 1 0 1; do
  GSPLAT_HIP_SSIM_FUSED=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_f$f.$RANDOM.json 2>/dev/null || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 3
exit 0
