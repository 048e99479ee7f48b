#!/bin/bash
# Round-5 batch 10: DP-path capture tests, full GPU suite + M2 bench/profile,
# SSIM channel-group A/B, DP-path bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5_b10; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_graph.py \
  tests/test_gpu_surfel.py -x -v --timeout 200 --timeout-method thread \
  -k "dp_step or gshard_rccl or 2dgs or surfel or Surfel" > $O/dp_tests.log 2>&1
rc=$?; echo "dp tests rc=$rc"; tail -4 $O/dp_tests.log; [ $rc -eq 0 ] || exit $rc
GSPLAT_HIP_SSIM_CPW=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q \
  -k "ssim or loss" --timeout 200 --timeout-method thread > $O/cpw1_tests.log 2>&1
rc=$?; echo "cpw1 tests rc=$rc"; tail -2 $O/cpw1_tests.log; [ $rc -eq 0 ] || exit $rc
NB=2 PROF=1 bash tools/r5_run.sh r5_b10 || exit $?
for r in 1 2; do
  GSPLAT_HIP_SSIM_CPW=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-traffic \
    > $O/bench_cpw1.$r.json 2> $O/bench_cpw1.$r.err || exit 5
  python -c "import json; d=json.load(open('$O/bench_cpw1.$r.json')); print('cpw1', d['value'], d['ms_per_step'])"
done
for m in "" "--eager"; do
  timeout -k 10 300 python bench.py --dp-path --no-cpu-baseline --no-traffic $m \
    > $O/bench_dp$m.json 2> $O/bench_dp$m.err || exit 6
  python -c "import json; d=json.load(open('$O/bench_dp$m.json')); print('dp$m', d['value'], d['ms_per_step'], d.get('step_issue'))"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --config m5 --no-cpu-baseline --no-traffic \
    > $O/bench_m5.$r.json 2> $O/bench_m5.$r.err || exit 7
  python -c "import json; d=json.load(open('$O/bench_m5.$r.json')); print('m5', d['value'], d['ms_per_step'], d.get('step_issue'))"
done
exit 0
