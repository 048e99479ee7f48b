#!/bin/bash
# M5 (2DGS training step) with and without the tile culling of large surfels
# in the captured step's isect (rendering.TILE_CULL), alternating, plus the
# kernel statistics of the default.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-m5_cull}; mkdir -p $O
for r in 1 2; do
  for c in 1 0; do
    timeout -k 10 300 python -u -c "
import sys
sys.argv = ['bench.py', '--config', 'm5', '--no-cpu-baseline', '--no-traffic', '--steps', '30']
sys.path.insert(0, '.'); sys.path.insert(0, 'gsplat-triton_amd')
import gsplat_hip.rendering as r
r.TILE_CULL = bool($c)
import bench
bench.main()" > $O/bench_m5_cull${c}_$r.json 2> $O/bench_m5_cull${c}_$r.err || exit 2
    python -c "import json; d=json.load(open('$O/bench_m5_cull${c}_$r.json')); print('m5 cull $c run $r', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 4
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 26 30 > $O/kstats_m5.txt 2>&1; head -14 $O/kstats_m5.txt
exit 0
