#!/bin/bash
# Round-4 batch: GPU suite, M2 default twice, emulated 8-rank gshard step
# graph-replayed (twice) and eager, M3 graph vs eager, a kernel trace of the
# default M2 line, the memset diagnosis.  Test failures are reported; crashes / time limits end it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
dead() { [ $1 -eq 124 ] || [ $1 -eq 137 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -1 $O/tests.log
  dead $rc && exit $rc
fi
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2.$r.json 2> $O/m2.$r.err || exit 2
  echo "m2 run $r $(v $O/m2.$r.json)"
done
for r in 1 2; do
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
# last (it may fault, nothing runs after it): the round-3 memset nodes
# restored in the captured step, replays serialized
GSPLAT_HIP_MEMSET_NODES=1 GSPLAT_HIP_GRAPH_ALLOW_MEMSET=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 180 python -u tools/graph_diag.py memset > $O/memset_diag.log 2>&1
echo "memset diag rc=$?"; tail -12 $O/memset_diag.log
exit 0
