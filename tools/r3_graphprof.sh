#!/bin/bash
# Per-kernel times of the graph-replayed step against the eager step (M2),
# after the whole -m gpu suite.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_graphprof}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in graph eager; do
  flag=""; [ $m = eager ] && flag="--eager"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/$m -o run -- /usr/bin/python3 bench.py $flag --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/$m.json 2> $O/$m.err
  rc=$?; echo "prof $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
