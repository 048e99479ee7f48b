# Forward pair-unroll A/B (GSPLAT_HIP_FWD_UNROLL = 1/2/4 pairs per composite
# iteration) on the M2 bench, after the raster parity tests at each setting.
set -o pipefail
O=gpurun_out/${AB_TAG:-abu}; mkdir -p $O
for u in 1 2 4; do
  GSPLAT_HIP_FWD_UNROLL=$u timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_raster_dispatch.py -x -q --timeout 120 --timeout-method thread > $O/tests_u$u.log 2>&1 || exit 1
done
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for u in ${AB_U:-1 2 4 1 2 4}; do
  GSPLAT_HIP_FWD_UNROLL=$u timeout -k 10 200 $B --config ${AB_CFG:-m2} > $O/u$u.$RANDOM.json 2>>$O/err.log || exit 2
done
