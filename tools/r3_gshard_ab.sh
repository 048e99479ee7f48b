#!/bin/bash
# The gshard GPU tests, then the emulated 8-rank per-rank step (twice) and
# the one-GPU line beside it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_gshard_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gshard.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(round(d['value'],1), round(d['ms_per_step'],4))"; }
for v in ${EMU_VARS:-8 8b eager1 graph1}; do
  case $v in graph1) A="";; eager1) A="--eager";; *) A="--gshard-emulate ${v%b}";; esac
  timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline $A > $O/m2.$v.json 2> $O/m2.$v.err
  rc=$?; echo "m2 $v rc=$rc $(summ $O/m2.$v.json)"; [ $rc -eq 0 ] || { tail -5 $O/m2.$v.err; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/emu -o run -- /usr/bin/python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --gshard-emulate 8 > $O/emu_trace.log 2>&1 || exit 3
echo trace ok
