# Repeat the bench (default M2, no PMC / CPU baseline) after the raster tests.
# usage: REP_TAG=x REP_N=4 REP_CFG=m2 bash tools/bench_rep.sh [extra bench args]
set -o pipefail
O=gpurun_out/${REP_TAG:-rep}; mkdir -p $O
if [ -z "$REP_NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_raster_dispatch.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
for i in $(seq 1 ${REP_N:-4}); do
  timeout -k 10 200 python bench.py --steps ${REP_STEPS:-30} --warmup 5 --no-cpu-baseline --no-traffic --config ${REP_CFG:-m2} "$@" > $O/b$i.json 2>>$O/err.log || exit 2
done
