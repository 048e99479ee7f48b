#!/bin/bash
# Round-5 batch 14: surfel kernels at higher occupancy (capped VGPRs) at M5.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b14; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_graph.py -x -q --timeout 200 \
  --timeout-method thread -k "e2e or depth_to_normal or 2dgs or packed" > $O/sel.log 2>&1
rc=$?; echo "selected tests rc=$rc"; tail -2 $O/sel.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base f5 b4 f5b4; do
    case $v in
      base) E="";; f5) E="GSPLAT_HIP_SURFEL_FWD_WPE=5";; b4) E="GSPLAT_HIP_SURFEL_BWD_WPE=4";;
      f5b4) E="GSPLAT_HIP_SURFEL_FWD_WPE=5 GSPLAT_HIP_SURFEL_BWD_WPE=4";;
    esac
    env $E timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic > $O/m5_$v.$r.json 2> $O/m5_$v.$r.err || exit 7
    python -c "import json; d=json.load(open('$O/m5_$v.$r.json')); print('m5 $v', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  done
done
exit 0
