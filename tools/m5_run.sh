#!/bin/bash
# 2DGS (BASELINE configs[4]) on the GPU box: surfel parity tests, a kernel
# trace of the m5 bench workload and the m5 bench line.  Usage: bash tools/m5_run.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_surfel.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- /usr/bin/python3 bench.py --config m5 --steps 10 --warmup 3 --no-cpu-baseline --no-traffic > $OUT/trace.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --config m5 --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:---no-traffic} > $OUT/bench.json 2> $OUT/bench.err || exit 3
exit 0
