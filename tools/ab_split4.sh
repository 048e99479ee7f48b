#!/bin/bash
# One-launch split forward: raster/parity/graph tests, then M2 and M3 lines
# with the split adaptive (default), off (GSPLAT_HIP_FWD_SPLIT=0) and the
# HEAD library (ab_lib/base.so), alternately.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_split4}; mkdir -p $O
[ -n "$AB_NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_raster_dispatch.py tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(r['launch_ms'],4), round(r['bwd']['launch_ms'],4))"; }
B="python -u bench.py --no-traffic --no-cpu-baseline"
for cfg in ${AB_CFGS:-m2 m3}; do
  for r in 1 2; do
    for v in ${AB_VARS:-split nosplit}; do
      unset GSPLAT_HIP_LIB GSPLAT_HIP_FWD_SPLIT
      [ $v = base ] && export GSPLAT_HIP_LIB=$PWD/ab_lib/base.so
      [ $v = nosplit ] && export GSPLAT_HIP_FWD_SPLIT=0
      timeout -k 10 300 $B --config $cfg > $O/$cfg.$v.$r.json 2> $O/$cfg.$v.$r.err
      rc=$?; echo "$cfg $v $r rc=$rc $(summ $O/$cfg.$v.$r.json)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
