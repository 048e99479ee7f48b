#!/bin/bash
# Geometry update with the activation VJPs / means sum folded in: trainer
# GPU tests, M2 bench off / on x2.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/geom; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for f in 0 1; do
    GSPLAT_HIP_GEOM_FUSE=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_f$f.$r.json 2>/dev/null || exit 2
  done
done
exit 0
