#!/bin/bash
# Backward pixels per lane with the per-strip pair skip: PX 2 (default) vs 4,
# parity tests under PX 4 first, then the M2 line alternately.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_bwdpx}; mkdir -p $O
GSPLAT_HIP_BWD_PX=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $O/tests_px4.log 2>&1
rc=$?; echo "tests px4 rc=$rc"; tail -2 $O/tests_px4.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for px in 2 4; do
    GSPLAT_HIP_BWD_PX=$px timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/px$px.$r.json 2> $O/px$px.$r.err
    rc=$?; echo "px$px $r rc=$rc $(python3 -c "import json;d=json.loads(open('$O/px$px.$r.json').read().strip().splitlines()[-1]);print(round(d['value'],1), round(d['roofline']['launch_ms'],4), round(d['roofline']['bwd']['launch_ms'],4))")"; [ $rc -eq 0 ] || exit $rc
  done
done
