#!/bin/bash
# One GPU-box session: the -m gpu suite, then the benches.  Each GPU step has
# its own time limit; after a crash / abort / time limit nothing else runs.
# usage: tools/gpu_round.sh TAG [bench args for the m2 line...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-run}; shift
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pytest: 1 = test failures, not a fault
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
  ok $rc || exit $rc
fi
timeout -k 10 420 python -u bench.py "$@" > gpurun_out/${TAG}_bench_m2.json 2> gpurun_out/${TAG}_bench_m2.err
rc=$?; echo "bench m2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_M3" ]; then
  timeout -k 10 300 python -u bench.py --config m3 --no-traffic --no-cpu-baseline \
    > gpurun_out/${TAG}_bench_m3.json 2> gpurun_out/${TAG}_bench_m3.err
  rc=$?; echo "bench m3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
