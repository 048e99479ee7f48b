#!/bin/bash
# Gaussian-sharded training at world 2 on one GPU (gloo), the whole -m gpu
# suite, the M2 line, and the VALU issue micro-benchmark.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_gshard}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gshard.py -x -v --timeout 300 --timeout-method thread > $O/gshard_tests.log 2>&1
rc=$?; echo "gshard tests rc=$rc"; tail -5 $O/gshard_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc $(tail -c 300 $O/bench.json)"; [ $rc -eq 0 ] || exit $rc
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/valu_bench.hip -o /tmp/valu_bench && timeout -k 10 60 /tmp/valu_bench > $O/valu_bench.txt 2>&1
echo "valu rc=$?"; cat $O/valu_bench.txt
