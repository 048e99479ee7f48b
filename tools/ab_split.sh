# Split-forward A/B (GSPLAT_HIP_FWD_SPLIT = 0 off / 1024 default / others) on M2 and M3,
# after the raster tests.
set -o pipefail
O=gpurun_out/${AB_TAG:-absplit}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster_dispatch.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for cfg in ${AB_CFGS:-m2 m3}; do
  for sp in ${AB_SP:--1 0 -1 0}; do
    GSPLAT_HIP_FWD_SPLIT=$sp timeout -k 10 200 $B --config $cfg > $O/$cfg.s$sp.$RANDOM.json 2>>$O/err.log || exit 2
  done
done
