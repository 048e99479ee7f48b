# Backward chunk length (GSPLAT_HIP_CHUNK) A/B on the M2 bench.
set -o pipefail
O=gpurun_out/${AB_TAG:-abchunk}; mkdir -p $O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic --config ${AB_CFG:-m2}"
for L in ${AB_L:-256 192 320 384 256 192 320}; do
  GSPLAT_HIP_CHUNK=$L timeout -k 10 200 $B > $O/L$L.$RANDOM.json 2>>$O/err.log || exit 2
done
