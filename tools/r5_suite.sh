#!/bin/bash
# The whole GPU suite and one default bench line (end-of-round check).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > $O/m2.json 2> $O/m2.err || exit 3
python -c "import json; d=json.load(open('$O/m2.json')); print('m2', round(d['value'],1), round(d['ms_per_step'],4))"
