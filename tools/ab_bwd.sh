# A/B of the backward's pixels-per-lane (GSPLAT_HIP_BWD_PX) on the M2 bench.
set -o pipefail
O=gpurun_out/${AB_TAG:-ab2}; mkdir -p $O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic"
GSPLAT_HIP_BWD_PX=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $O/tests_px4.log 2>&1 || exit 1
for px in 2 4 1 2 4; do
  GSPLAT_HIP_BWD_PX=$px timeout -k 10 200 $B > $O/px$px.$RANDOM.json 2>>$O/err.log || exit 2
done
GSPLAT_HIP_BWD_PX=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace4 -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace4.log 2>&1 || exit 6
