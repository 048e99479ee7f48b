# 3DGS forward A/B (GSPLAT_HIP_FWD_UNROLL=2: pair loop unrolled 1/2/4 times) on the M2 bench, after the parity tests.
set -o pipefail
O=gpurun_out/${AB_TAG:-abf}; mkdir -p $O
GSPLAT_HIP_FWD_UNROLL=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trainer.py tests/test_gpu_indices.py tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic"
for px in 4 2 4 2; do
  GSPLAT_HIP_FWD_UNROLL=$px timeout -k 10 200 $B > $O/fpx$px.$RANDOM.json 2>>$O/err.log || exit 2
done
