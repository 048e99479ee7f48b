#!/bin/bash
# A/B of the working-tree library against ab_lib/base.so (built from HEAD):
# GPU parity tests on the new library, then the M2 line alternately, then
# the new library's line with PMC traffic.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_lib}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(r['launch_ms'],4), round(r['bwd']['launch_ms'],4), r.get('traffic'), r['bwd'].get('traffic'))"; }
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export GSPLAT_HIP_LIB=$PWD/ab_lib/base.so; else unset GSPLAT_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/$v.$r.json 2> $O/$v.$r.err
    rc=$?; echo "$v $r rc=$rc $(summ $O/$v.$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
unset GSPLAT_HIP_LIB
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/new.traffic.json 2> $O/new.traffic.err
rc=$?; echo "new traffic rc=$rc $(summ $O/new.traffic.json)"; exit $rc
