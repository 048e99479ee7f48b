#!/bin/bash
# Round evidence: the -m gpu suite, the default bench line (PMC traffic + CPU
# baseline), rocprofv3 kernel stats of the M2 bench, then the M3 and M5 lines.
# Each GPU step has its own time limit; after a failure nothing else runs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:-final}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench_m2.json 2> $O/bench_m2.err || exit 2
echo "bench m2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 3
echo "trace ok"
timeout -k 10 300 python -u bench.py --config m3 --no-traffic --no-cpu-baseline > $O/bench_m3.json 2> $O/bench_m3.err || exit 4
timeout -k 10 300 python -u bench.py --config m5 --no-traffic --no-cpu-baseline > $O/bench_m5.json 2> $O/bench_m5.err || exit 5
echo "m3 m5 ok"
exit 0
