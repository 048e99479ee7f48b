#!/bin/bash
# Round-5 final evidence (profiles/r5/final, final2, final3 were made by its
# earlier forms): the whole GPU suite, the default bench line (PMC traffic + CPU baseline),
# its rocprofv3 kernel stats, the other configurations' lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_final3}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -1 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_m2.json 2> $O/bench_m2.err || exit 3
python -c "import json; d=json.load(open('$O/bench_m2.json')); print('m2', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['traffic'], 'cpu', d['cpu_baseline'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m2 -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace_m2.log 2>&1 || exit 4
python tools/kstats.py $(find $O/trace_m2 -name "*kernel_stats.csv" | head -1) 26 30 > $O/kstats_m2.txt 2>&1; head -12 $O/kstats_m2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 4
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 26 30 > $O/kstats_m5.txt 2>&1; head -8 $O/kstats_m5.txt
for c in m5 m3; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', round(d['value'],1), round(d['ms_per_step'],4), d['roofline']['launch_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --gshard-emulate 8 --no-cpu-baseline --no-traffic > $O/bench_gs8.json 2> $O/bench_gs8.err || exit 6
python -c "import json; d=json.load(open('$O/bench_gs8.json')); print('gs8', round(d['value'],1), round(d['ms_per_step'],4), d.get('step_issue'))"
timeout -k 10 300 python bench.py --dp-emulate 8 --no-cpu-baseline --no-traffic > $O/bench_dp8.json 2> $O/bench_dp8.err || exit 6
python -c "import json; d=json.load(open('$O/bench_dp8.json')); print('dp8', round(d['value'],1), round(d['ms_per_step'],4), d.get('step_issue'))"
exit 0
