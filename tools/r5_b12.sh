#!/bin/bash
# Round-5 batch 12: surfel tile order A/B at M5, then the full GPU suite and
# the default M2 / M3 / M5 bench lines with kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b12; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_distributed.py -x -v --timeout 200 \
  --timeout-method thread -k "order or records or dp_step" > $O/sel.log 2>&1
rc=$?; echo "selected tests rc=$rc"; tail -2 $O/sel.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    GSPLAT_HIP_SURFEL_ORDER=$v timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic > $O/m5_o$v.$r.json 2> $O/m5_o$v.$r.err || exit 7
    python -c "import json; d=json.load(open('$O/m5_o$v.$r.json')); print('m5 order=$v', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  done
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
exit $rc
