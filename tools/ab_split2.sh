# Split-forward chunk length A/B: GSPLAT_HIP_FWD_SPLIT_CHUNK (with the
# adaptive threshold) against the split off, M2 and M3.
set -o pipefail
O=gpurun_out/${AB_TAG:-absc}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster_dispatch.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for cfg in ${AB_CFGS:-m2 m3}; do
  for v in ${AB_V:-256 512 off 256 512 off}; do
    if [ "$v" = off ]; then sp=0; sc=1024; else sp=-1; sc=$v; fi
    GSPLAT_HIP_FWD_SPLIT=$sp GSPLAT_HIP_FWD_SPLIT_CHUNK=$sc timeout -k 10 200 $B --config $cfg > $O/$cfg.c$v.$RANDOM.json 2>>$O/err.log || exit 2
  done
done
