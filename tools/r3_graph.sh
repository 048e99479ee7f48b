#!/bin/bash
# Graph-replayed step: its tests first, then the whole -m gpu suite, then the
# M2 line replayed (default) and eager (--eager), back to back on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_graph}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread > $O/graph_tests.log 2>&1
rc=$?; echo "graph tests rc=$rc"; tail -3 $O/graph_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/bench_graph.json 2> $O/bench_graph.err
rc=$?; echo "bench graph rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --eager --no-traffic --no-cpu-baseline > $O/bench_eager.json 2> $O/bench_eager.err
rc=$?; echo "bench eager rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --dp-emulate 8 --no-traffic --no-cpu-baseline > $O/bench_dp8.json 2> $O/bench_dp8.err
rc=$?; echo "bench dp8 rc=$rc"; exit $rc
