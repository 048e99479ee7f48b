#!/bin/bash
# Quick GPU check of a change: trainer + parity GPU tests, two M2 bench lines,
# rocprofv3 kernel stats of the M2 bench.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench.$r.json 2>/dev/null || exit 2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 3
exit 0
