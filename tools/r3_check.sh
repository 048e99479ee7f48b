#!/bin/bash
# The whole -m gpu suite, then the default M2 line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(round(d['value'],1), round(d['roofline']['launch_ms'],4), round(d['roofline']['bwd']['launch_ms'],4))")"
exit $rc
