#!/bin/bash
# Fused SSIM variants: loss fwd+bwd microbench, kernel stats per variant.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${AB_TAG:-ssimf2}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_trainer.py -x -q -k "ssim or fused_loss" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/ssim_bench.py 0 >> $O/micro.txt 2>&1 || exit 2
for v in 0 1; do
  GSPLAT_HIP_SSIM_FV=$v timeout -k 10 120 python -u tools/ssim_bench.py 1 >> $O/micro.txt 2>&1 || exit 3
  GSPLAT_HIP_SSIM_FV=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/v$v -o run -- /usr/bin/python3 tools/ssim_bench.py 1 > /dev/null 2>&1 || exit 4
done
cat $O/micro.txt
exit 0
