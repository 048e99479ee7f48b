#!/bin/bash
# M5 (2DGS training step): two bench lines and the kernel statistics.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-m5}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config m5 --no-cpu-baseline --no-traffic --steps 30 \
    > $O/bench_m5_$r.json 2> $O/bench_m5_$r.err || exit 2
  python -c "import json; d=json.load(open('$O/bench_m5_$r.json')); print('m5 run $r', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 4
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 26 30 > $O/kstats_m5.txt 2>&1; head -8 $O/kstats_m5.txt
exit 0
