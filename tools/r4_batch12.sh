#!/bin/bash
# Round-4 batch 12: the geometry Adam non-temporal (GSPLAT_HIP_ADAM_NT) A/B at
# M2, alternating; Adam / trainer / graph tests under NT=1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch12}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
GSPLAT_HIP_ADAM_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_graph.py -q --timeout 180 --timeout-method thread > $O/tests_nt.log 2>&1
rc=$?; echo "tests (ADAM_NT=1) rc=$rc"; grep FAILED $O/tests_nt.log; tail -1 $O/tests_nt.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for nt in 0 1; do
    GSPLAT_HIP_ADAM_NT=$nt timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2_nt$nt.$r.json 2> $O/m2_nt$nt.$r.err || exit 2
    echo "m2 adam_nt=$nt run $r $(v $O/m2_nt$nt.$r.json)"
  done
done
