#!/bin/bash
# HEAD validation on one MI355X: the whole GPU suite, smoke, then M2 / M3
# lines with the default (adaptive device-side split) and the split off
# (noovl: GSPLAT_HIP_ISECT_OVERLAP=0, a switch of a reverted experiment).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_validate}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(r['launch_ms'],4), round(r['bwd']['launch_ms'],4))"; }
for cfg in ${AB_CFGS:-m2 m3}; do
  for r in 1 2; do
    for v in ${AB_VARS:-default nosplit}; do
      unset GSPLAT_HIP_FWD_SPLIT GSPLAT_HIP_ISECT_OVERLAP
      [ $v = nosplit ] && export GSPLAT_HIP_FWD_SPLIT=0
      [ $v = noovl ] && export GSPLAT_HIP_ISECT_OVERLAP=0
      timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline --config $cfg > $O/$cfg.$v.$r.json 2> $O/$cfg.$v.$r.err
      rc=$?; echo "$cfg $v $r rc=$rc $(summ $O/$cfg.$v.$r.json)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
