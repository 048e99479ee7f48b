#!/bin/bash
# Round-end evidence on one GPU box.  Part "a": the whole -m gpu suite, the
# default bench line (PMC traffic + CPU baseline) and the kernel statistics of
# the same workload.  Part "b": the M3 / M5 lines with PMC traffic, the M5
# kernel statistics, the one-GPU line with the data-parallel phase and the
# emulated 8-rank per-rank steps.  Every GPU step has its own time limit;
# after a fault, abort or time limit nothing else runs.
# usage: tools/final_r6.sh TAG a|b
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p $O
line() { python -c "import json,sys; d=json.load(open('$1')); r=d.get('roofline',{}); print('$2', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', r.get('launch_ms'), 'bwd', (r.get('bwd') or {}).get('launch_ms'), 'traffic', r.get('traffic'))"; }
if [ "$2" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
    > $O/suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 600 python -u bench.py > $O/bench_m2.json 2> $O/bench_m2.err || exit 2
  line $O/bench_m2.json m2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m2 -o run -- \
    /usr/bin/python3 bench.py --no-cpu-baseline --no-traffic > $O/trace_m2.log 2>&1 || exit 3
  python tools/kstats.py $(find $O/trace_m2 -name "*kernel_stats.csv" | head -1) 35 30 > $O/kstats_m2.txt 2>&1
  head -12 $O/kstats_m2.txt
  exit $rc
fi
timeout -k 10 400 python -u bench.py --config m3 --no-cpu-baseline > $O/bench_m3.json 2> $O/bench_m3.err || exit 4
line $O/bench_m3.json m3
timeout -k 10 400 python -u bench.py --config m5 --no-cpu-baseline > $O/bench_m5.json 2> $O/bench_m5.err || exit 5
line $O/bench_m5.json m5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- \
  /usr/bin/python3 bench.py --config m5 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 6
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 35 30 > $O/kstats_m5.txt 2>&1
head -8 $O/kstats_m5.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --dp-phase > $O/bench_dpphase.json 2> $O/bench_dpphase.err || exit 7
python -c "import json; d=json.load(open('$O/bench_dpphase.json')); print('m2', round(d['value'],1), 'dp', {k: d['config']['dp'].get(k) for k in ('value', 'ms_per_step', 'error')})"
timeout -k 10 300 python -u bench.py --gshard-emulate 8 --no-cpu-baseline --no-traffic > $O/bench_gs8.json 2> $O/bench_gs8.err || exit 8
line $O/bench_gs8.json gs8
timeout -k 10 300 python -u bench.py --dp-path --dp-emulate 8 --no-cpu-baseline --no-traffic > $O/bench_dp8.json 2> $O/bench_dp8.err || exit 9
line $O/bench_dp8.json dp8
exit 0
