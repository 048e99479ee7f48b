#!/bin/bash
# Backward record prefetch (GSPLAT_HIP_BWD_PF) x pixels per lane: parity
# tests with the prefetch on, then M2 bench lines (bwd launch time).
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/bwdpf; mkdir -p $O
GSPLAT_HIP_BWD_PF=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_raster_dispatch.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for cfg in "4 0" "4 1" "2 0" "2 1"; do
    set -- $cfg
    GSPLAT_HIP_BWD_PX=$1 GSPLAT_HIP_BWD_PF=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_px$1_pf$2.$r.json 2>/dev/null || exit 2
  done
done
exit 0
