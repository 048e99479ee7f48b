#!/bin/bash
# Round-5 batch 11: scalar-record surfel backward (and its 4-wave variant) vs
# the LDS-queue backward at M5; the full GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b11; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_graph.py -x -v --timeout 200 \
  --timeout-method thread -k "records or 2dgs or e2e" > $O/sel.log 2>&1
rc=$?; echo "selected tests rc=$rc"; tail -2 $O/sel.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "base" "bwd" "bwdw4"; do
    case $v in
      base) E="";; bwd) E="GSPLAT_HIP_SURFEL_SREC_BWD=1";; bwdw4) E="GSPLAT_HIP_SURFEL_SREC_BWD=1 GSPLAT_HIP_SURFEL_BWD_W4=1";;
    esac
    env $E timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic > $O/m5_$v.$r.json 2> $O/m5_$v.$r.err || exit 7
    python -c "import json; d=json.load(open('$O/m5_$v.$r.json')); print('m5 $v', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
exit $rc
