#!/bin/bash
# A/B of one environment switch inside the same library (no second .so):
#   tools/ab_env.sh TAG VAR "VALUE_A VALUE_B" [bench args...]
# GPU parity suite first (unless SKIP_TESTS), then the M2 line alternately
# A, B, A, B, then (unless SKIP_TRACE) a kernel trace of the B setting.
# Each GPU step has its own time limit; after a failure nothing else runs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1; VAR=$2; VALS=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline "$@" > $O/$v.$r.json 2> $O/$v.$r.err
    rc=$?; echo "$VAR=$v run $r rc=$rc $(summ $O/$v.$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
if [ -z "$SKIP_TRACE" ]; then
  last=${VALS##* }
  export $VAR=$last
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic "$@" > $O/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
