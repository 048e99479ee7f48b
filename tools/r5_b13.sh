#!/bin/bash
# Round-5 batch 13: the full GPU suite, then the default bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b13; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; [ $rc -eq 0 ] || exit $rc
for c in m2 m5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-traffic > $O/bench_$c.json 2> $O/bench_$c.err || exit 7
  python -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4), d.get('step_issue'))"
done
exit 0
