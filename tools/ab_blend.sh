#!/bin/bash
# Forward blend form A/B (GSPLAT_HIP_FWD_BLEND 0: masks combined on the SALU,
# 1: each select on its compare's mask): parity under 1, then M2 and M3 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_blend}; mkdir -p $O
GSPLAT_HIP_FWD_BLEND=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_raster_dispatch.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/tests_b1.log 2>&1
rc=$?; echo "tests b1 rc=$rc"; tail -2 $O/tests_b1.log; [ $rc -eq 0 ] || exit $rc
for cfg in m2 m3; do
  for r in 1 2; do
    for b in 0 1; do
      GSPLAT_HIP_FWD_BLEND=$b timeout -k 10 300 python -u bench.py --config $cfg --no-traffic --no-cpu-baseline > $O/$cfg.b$b.$r.json 2> $O/$cfg.b$b.$r.err
      rc=$?; echo "$cfg b$b $r rc=$rc $(python3 -c "import json;d=json.loads(open('$O/$cfg.b$b.$r.json').read().strip().splitlines()[-1]);print(round(d['value'],1), round(d['roofline']['launch_ms'],4), round(d['roofline']['bwd']['launch_ms'],4))")"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
