#!/bin/bash
# Round-4 batch 10: the whole GPU suite (incl. the split-divisor test), the
# SH Adam rows non-temporal A/B at M2 (GSPLAT_HIP_SH_ADAM_NT, alternating),
# M3 eager with the trainer-chosen divisor against a forced 550, a kernel
# trace of the default M2 workload.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch10}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];c=d['config'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'div', c.get('fwd_split_div'), 'ratio', c.get('termination_ratio_first_render'))"; }
dead() { [ $1 -eq 124 ] || [ $1 -eq 137 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -1 $O/tests.log
dead $rc && exit $rc
for r in 1 2; do
  for nt in 0 1; do
    GSPLAT_HIP_SH_ADAM_NT=$nt timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2_nt$nt.$r.json 2> $O/m2_nt$nt.$r.err || exit 2
    echo "m2 nt=$nt run $r $(v $O/m2_nt$nt.$r.json)"
  done
done
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config m3 --eager --no-traffic --no-cpu-baseline > $O/m3_auto.$r.json 2> $O/m3_auto.$r.err || exit 3
  echo "m3 eager auto run $r $(v $O/m3_auto.$r.json)"
  GSPLAT_HIP_FWD_SPLIT_DIV=550 timeout -k 10 400 python -u bench.py --config m3 --eager --no-traffic --no-cpu-baseline > $O/m3_550.$r.json 2> $O/m3_550.$r.err || exit 4
  echo "m3 eager div550 run $r $(v $O/m3_550.$r.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 6
echo "trace ok"
