#!/bin/bash
# Round-5 batch 10: 2DGS / data-parallel capture tests, scalar-record forward
# A/B (surfel and 3DGS), M5 counters and kernel stats, SSIM channel-group A/B.
# The data-parallel capture with RCCL collectives runs last (its previous
# form crashed in hipStreamEndCapture).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b10; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py \
  tests/test_gpu_surfel.py tests/test_gpu_raster_dispatch.py -x -v --timeout 200 --timeout-method thread \
  -k "(dp_step and 1-None) or 2dgs or scalar_record or records_bit" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline $([ $r = 2 ] && echo --no-traffic) \
    > $O/bench_m5.$r.json 2> $O/bench_m5.$r.err || exit 7
  python -c "import json; d=json.load(open('$O/bench_m5.$r.json')); print('m5', d['value'], d['ms_per_step'], d.get('step_issue'), d['roofline'].get('launch_ms'), d['roofline'].get('bwd',{}).get('launch_ms'))"
  GSPLAT_HIP_SURFEL_SREC=1 timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic \
    > $O/bench_m5_srec.$r.json 2> $O/bench_m5_srec.$r.err || exit 9
  python -c "import json; d=json.load(open('$O/bench_m5_srec.$r.json')); print('m5 srec', d['value'], d['ms_per_step'], d['roofline'].get('launch_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m5 -o run -- /usr/bin/python3 bench.py --config m5 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $O/trace_m5.log 2>&1 || exit 8
python tools/kstats.py $(find $O/trace_m5 -name "*kernel_stats.csv" | head -1) 13 > $O/kstats_m5.txt 2>&1; head -22 $O/kstats_m5.txt
for r in 1 2; do
  GSPLAT_HIP_FWD_SREC=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic \
    > $O/bench_fsrec.$r.json 2> $O/bench_fsrec.$r.err || exit 10
  python -c "import json; d=json.load(open('$O/bench_fsrec.$r.json')); print('fwd srec', d['value'], d['ms_per_step'], d['roofline'].get('launch_ms'))"
  for cpw in 3 1; do
    GSPLAT_HIP_SSIM_CPW=$cpw timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic \
      > $O/bench_cpw$cpw.$r.json 2> $O/bench_cpw$cpw.$r.err || exit 5
    python -c "import json; d=json.load(open('$O/bench_cpw$cpw.$r.json')); print('cpw$cpw', d['value'], d['ms_per_step'], d['roofline'].get('launch_ms'))"
  done
done
for m in "" "--eager"; do
  timeout -k 10 300 python bench.py --dp-path --no-cpu-baseline --no-traffic $m \
    > $O/bench_dp$m.json 2> $O/bench_dp$m.err || exit 6
  python -c "import json; d=json.load(open('$O/bench_dp$m.json')); print('dp$m', d['value'], d['ms_per_step'], d.get('step_issue'))"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
  -k "dp_step" > $O/dp_tests.log 2>&1
rc=$?; echo "dp tests rc=$rc"; tail -4 $O/dp_tests.log
exit $rc
