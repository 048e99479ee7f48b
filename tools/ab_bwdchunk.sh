#!/bin/bash
# Backward chunk length (GSPLAT_HIP_CHUNK) with the PX=2 + prefetch default,
# and the one-pixel kernel for reference: M2 bench lines.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/bwdchunk; mkdir -p $O
for r in 1 2; do
  for L in 128 192 256 384; do
    GSPLAT_HIP_CHUNK=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_L$L.$r.json 2>/dev/null || exit 2
  done
  GSPLAT_HIP_BWD_PX=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_px1.$r.json 2>/dev/null || exit 3
done
exit 0
