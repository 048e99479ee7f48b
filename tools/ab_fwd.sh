# Forward A/B: register budget (GSPLAT_HIP_FWD_OCC 5/6) on the M2 bench, after the parity tests.
set -o pipefail
O=gpurun_out/${AB_TAG:-abf1}; mkdir -p $O
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trainer.py tests/test_gpu_indices.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
GSPLAT_HIP_FWD_OCC=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests5.log 2>&1 || exit 1
for o in 6 5 6 5; do
  GSPLAT_HIP_FWD_OCC=$o timeout -k 10 200 $B > $O/occ$o.$RANDOM.json 2>>$O/err.log || exit 2
done
for o in 6 5; do
  GSPLAT_HIP_FWD_OCC=$o timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace$o -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace$o.log 2>&1 || exit 6
done
