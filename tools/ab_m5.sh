#!/bin/bash
# M5 (2DGS) with the SH groups' Adam fused into the SH backward off / on,
# after the 2DGS GPU tests.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/m5shadam; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_fit.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    GSPLAT_HIP_SH_ADAM_IN_BWD=$f timeout -k 10 300 python -u bench.py --config m5 --no-cpu-baseline --no-traffic > $O/bench_f$f.$r.json 2>/dev/null || exit 2
  done
done
exit 0
