#!/bin/bash
# Round-5 batch 18: the fused loss on the RGB+D render in place (2DGS): loss
# tests, 2DGS / graph tests, M5 lines; then M2 to check the 3DGS loss path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_graph.py tests/test_gpu_surfel.py \
  tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread \
  -k "loss or ssim or 2dgs or graph or e2e or sharded" > $O/sel.log 2>&1
rc=$?; echo "selected tests rc=$rc"; tail -2 $O/sel.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic > $O/m5.$r.json 2> $O/m5.$r.err || exit 7
  python -c "import json; d=json.load(open('$O/m5.$r.json')); print('m5', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic > $O/m2.json 2> $O/m2.err || exit 7
python -c "import json; d=json.load(open('$O/m2.json')); print('m2', round(d['value'],1), round(d['ms_per_step'],4))"
