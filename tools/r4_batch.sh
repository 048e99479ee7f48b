#!/bin/bash
# Round-4 batch: GPU suite, lazy SH Adam / side-stream SH / SH-Adam unroll / one-launch depth sort A/B (M2), emulated 8-rank gshard
# step graph vs eager, M3 graph vs eager, a kernel trace of the default M2
# line, and last the memset diagnosis (it may fault: nothing runs after it).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -2 $O/tests.log
  # failures are reported, crashes / time limits end the call
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
fi
# the one-launch depth sort (GSPLAT_HIP_DSORT=1): the isect / graph tests with it
GSPLAT_HIP_DSORT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 180 --timeout-method thread > $O/tests_dsort.log 2>&1
drc=$?; echo "dsort tests rc=$drc"; tail -2 $O/tests_dsort.log
[ $drc -eq 124 ] || [ $drc -eq 137 ] || [ $drc -eq 134 ] || [ $drc -eq 139 ] && exit 7
for r in 1 2; do
  for c in "0 0 4 0" "0 0 1 0" "1 0 4 0" "0 1 4 0" "0 0 4 1"; do
    set -- $c
    [ $4 = 1 ] && [ $drc -ne 0 ] && continue
    n=m2_lazy$1_side$2_u$3_ds$4.$r
    GSPLAT_HIP_SH_LAZY=$1 GSPLAT_HIP_SIDE_SH=$2 GSPLAT_HIP_SH_ADAM_U=$3 GSPLAT_HIP_DSORT=$4 timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/$n.json 2> $O/$n.err || exit 2
    echo "m2 lazy=$1 side=$2 adam_u=$3 dsort=$4 run $r $(v $O/$n.json)"
  done
done
for r in 1; do
  timeout -k 10 400 python -u bench.py --gshard-emulate 8 --no-traffic --no-cpu-baseline > $O/gs8_graph.$r.json 2> $O/gs8_graph.$r.err || exit 3
  echo "gshard-emulate 8 graph run $r $(v $O/gs8_graph.$r.json)"
done
timeout -k 10 400 python -u bench.py --gshard-emulate 8 --eager --no-traffic --no-cpu-baseline > $O/gs8_eager.json 2> $O/gs8_eager.err || exit 4
echo "gshard-emulate 8 eager $(v $O/gs8_eager.json)"
for m in graph eager; do
  a=""; [ $m = eager ] && a="--eager"
  timeout -k 10 400 python -u bench.py --config m3 --no-traffic --no-cpu-baseline $a > $O/m3_$m.json 2> $O/m3_$m.err || exit 5
  echo "m3 $m $(v $O/m3_$m.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 6
echo "trace ok"
if [ -n "$MEMSET_DIAG" ]; then
  GSPLAT_HIP_MEMSET_NODES=1 GSPLAT_HIP_GRAPH_ALLOW_MEMSET=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 180 python -u tools/graph_diag.py memset > $O/memset_diag.log 2>&1
  echo "memset diag rc=$?"; tail -5 $O/memset_diag.log
fi
exit 0
