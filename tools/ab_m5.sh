# 2DGS rasterizer A/B on the M5 bench (GSPLAT_HIP_FWD_PX / GSPLAT_HIP_BWD_PX = 1: one pixel per
# lane), after the surfel parity tests.
set -o pipefail
O=gpurun_out/${AB_TAG:-abm5}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_fit.py tests/test_gpu_indices.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --config m5 --steps 15 --warmup 3 --no-cpu-baseline --no-traffic"
for px in 2 1 2 1; do
  GSPLAT_HIP_FWD_PX=$px timeout -k 10 200 $B > $O/fpx$px.$RANDOM.json 2>>$O/err.log || exit 2
done
