#!/bin/bash
# New GPU tests of this round, then the M2 line of the N>1 code path on a
# 1-rank RCCL group (--dp-path) and the default M2 line, back to back.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_dp}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multicam.py tests/test_gpu_parity.py tests/test_gpu_trainer.py tests/test_gpu_strategy.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --dp-path --no-traffic --no-cpu-baseline > $O/bench_dp.json 2> $O/bench_dp.err
rc=$?; echo "bench dp rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/bench_m2.json 2> $O/bench_m2.err
rc=$?; echo "bench m2 rc=$rc"; exit $rc
