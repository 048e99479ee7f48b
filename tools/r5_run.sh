#!/bin/bash
# Round-5 GPU session: selected / all GPU tests, M2 bench lines, kernel stats.
# usage: tools/r5_run.sh TAG [TESTS...]   (TESTS default: the whole -m gpu suite)
# env: NB (bench lines, default 2), PROF=1 (rocprofv3 kernel stats of M2),
#      BENCH_ARGS (extra bench.py args), SKIP_TESTS=1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r5}; shift
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  T=${@:-tests}
  timeout -k 10 1000 python -u -m pytest $T -m gpu -x -v --timeout 150 --timeout-method thread \
    > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${NB:-2}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic $BENCH_ARGS > $O/bench.$r.json 2> $O/bench.$r.err
  rc=$?; echo "bench $r rc=$rc $(python -c "import json,sys; d=json.load(open('$O/bench.$r.json')); print(round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))" 2>&1)"
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic $BENCH_ARGS > $O/trace.log 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/kstats.py $(find $O/trace -name "*kernel_stats.csv" | head -1) 46 > $O/kstats.txt 2>&1; head -40 $O/kstats.txt
fi
exit 0
