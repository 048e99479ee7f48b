#!/bin/bash
# Kernel trace of the emulated 8-rank Gaussian-sharded step (one GPU) and of
# the one-GPU eager step, for tools/step_timeline.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_gshard_prof}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gshard.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline --gshard-emulate 8 > $O/emu8.json 2> $O/emu8.err || exit 2
python3 -c "import json;d=json.loads(open('$O/emu8.json').read().strip().splitlines()[-1]);print('emu8', round(d['value'],1), round(d['ms_per_step'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/emu -o run -- /usr/bin/python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --gshard-emulate 8 > $O/emu_trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/eager -o run -- /usr/bin/python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --eager > $O/eager_trace.log 2>&1 || exit 4
echo traces ok
