# Forward gather prefetch A/B (GSPLAT_HIP_FWD_PF = 1: double-buffered
# attributes, 5 waves/SIMD; 0: single buffer, 7 waves/SIMD) on M2 and M3.
set -o pipefail
O=gpurun_out/${AB_TAG:-abpf}; mkdir -p $O
for pf in ${AB_PFT:-0 1}; do
  GSPLAT_HIP_FWD_PF=$pf timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_raster_dispatch.py -x -q --timeout 120 --timeout-method thread > $O/tests_pf$pf.log 2>&1 || exit 1
done
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for cfg in m2 m3; do
  for pf in ${AB_PF:-0 1 0 1}; do
    GSPLAT_HIP_FWD_PF=$pf timeout -k 10 200 $B --config $cfg > $O/$cfg.pf$pf.$RANDOM.json 2>>$O/err.log || exit 2
  done
done
