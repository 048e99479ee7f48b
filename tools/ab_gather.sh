# Rasterizer gather A/B: render records (GSPLAT_HIP_RECORDS) x XCD-aware
# dispatch (GSPLAT_HIP_XCD) on the M2 and M3 benches, after the raster tests.
set -o pipefail
O=gpurun_out/${AB_TAG:-abg}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster_dispatch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for cfg in m2 m3; do
  for rx in ${AB_RX:-11 00 10 01}; do
    r=${rx:0:1}; x=${rx:1:1}
    GSPLAT_HIP_RECORDS=$r GSPLAT_HIP_XCD=$x timeout -k 10 240 $B --config $cfg > $O/$cfg.r$r.x$x.json 2>>$O/err.log || exit 2
  done
done
