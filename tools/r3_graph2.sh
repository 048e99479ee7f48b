#!/bin/bash
# Graph tests, the whole -m gpu suite, then the M2 line graph-replayed and
# eager alternately (box noise), then a kernel trace of the graph-replayed run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_graph2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread > $O/graph_tests.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -3 $O/graph_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for m in graph eager; do
    flag=""; [ $m = eager ] && flag="--eager"
    timeout -k 10 300 python -u bench.py $flag --no-traffic --no-cpu-baseline > $O/bench_$m.$r.json 2> $O/bench_$m.$r.err
    rc=$?; echo "bench $m $r rc=$rc $(python3 -c "import json;d=json.loads(open('$O/bench_$m.$r.json').read().strip().splitlines()[-1]);print(round(d['value'],1), round(d['ms_per_step'],4))")"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/graph -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/prof_graph.json 2> $O/prof_graph.err
echo "prof rc=$?"
