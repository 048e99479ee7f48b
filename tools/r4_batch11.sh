#!/bin/bash
# Round-4 batch 11: the trainer-chosen split divisor (termination ratio) --
# trainer / dispatch / graph tests, M3 eager with the auto divisor against a
# forced 550 (alternating), M2 auto (must keep 550).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch11}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];c=d['config'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'div', c.get('fwd_split_div'), 'ratio', c.get('termination_ratio_first_render'))"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_raster_dispatch.py tests/test_gpu_graph.py -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2.json 2> $O/m2.err || exit 2
echo "m2 auto $(v $O/m2.json)"
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config m3 --eager --no-traffic --no-cpu-baseline > $O/m3_auto.$r.json 2> $O/m3_auto.$r.err || exit 3
  echo "m3 eager auto run $r $(v $O/m3_auto.$r.json)"
  GSPLAT_HIP_FWD_SPLIT_DIV=550 timeout -k 10 400 python -u bench.py --config m3 --eager --no-traffic --no-cpu-baseline > $O/m3_550.$r.json 2> $O/m3_550.$r.err || exit 4
  echo "m3 eager div550 run $r $(v $O/m3_550.$r.json)"
done
