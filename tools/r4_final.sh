#!/bin/bash
# Round-4 final evidence: GPU suite, the default bench line as the driver runs
# it (PMC traffic + CPU baseline), a kernel trace of the default workload, M3
# eager + graph, M5, the emulated 8-rank Gaussian-sharded step (graph).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_final}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
dead() { [ $1 -eq 124 ] || [ $1 -eq 137 ] || [ $1 -eq 134 ] || [ $1 -eq 139 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -1 $O/tests.log
dead $rc && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_m2.json 2> $O/bench_m2.err || exit 2
echo "bench default $(v $O/bench_m2.json)"
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2.2.json 2> $O/m2.2.err || exit 3
echo "m2 run 2 $(v $O/m2.2.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 4
echo "trace ok"
for m in eager graph; do
  a=""; [ $m = eager ] && a="--eager"
  timeout -k 10 400 python -u bench.py --config m3 --no-traffic --no-cpu-baseline $a > $O/m3_$m.json 2> $O/m3_$m.err || exit 5
  echo "m3 $m $(v $O/m3_$m.json)"
done
timeout -k 10 300 python -u bench.py --config m5 --no-traffic --no-cpu-baseline > $O/bench_m5.json 2> $O/bench_m5.err || exit 6
echo "m5 $(v $O/bench_m5.json)"
timeout -k 10 400 python -u bench.py --gshard-emulate 8 --no-traffic --no-cpu-baseline > $O/gs8_graph.json 2> $O/gs8_graph.err || exit 7
echo "gshard-emulate 8 graph $(v $O/gs8_graph.json)"
