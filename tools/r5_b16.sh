#!/bin/bash
# Round-5 batch 16: visible-row records / gradient rows and the faster order
# kernel for the surfel rasterizer: 2DGS tests, M5 lines, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_surfel.py tests/test_gpu_graph.py tests/test_gpu_distributed.py \
  tests/test_gpu_strategy.py -x -q --timeout 200 --timeout-method thread -k "surfel or raster2dgs or 2dgs or e2e" > $O/sel.log 2>&1
rc=$?; echo "selected tests rc=$rc"; tail -2 $O/sel.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic > $O/m5.$r.json 2> $O/m5.$r.err || exit 7
  python -c "import json; d=json.load(open('$O/m5.$r.json')); print('m5', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 8
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 23 24 > $O/kstats_m5.txt 2>&1; cat $O/kstats_m5.txt
