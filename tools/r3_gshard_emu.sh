#!/bin/bash
# Per-rank step of the Gaussian-sharded multi-GPU path on one MI355X
# (bench.py --gshard-emulate W): the gshard GPU tests, then M2 lines for
# W = 2, 4, 8 and the one-GPU eager and graph lines beside them.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r3_gshard_emu}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gshard.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],4), round(r['launch_ms'],4), round(r['bwd']['launch_ms'],4))"; }
B="python -u bench.py --no-traffic --no-cpu-baseline"
for v in ${EMU_VARS:-8 4 2 eager1 graph1 8b}; do
  case $v in
    eager1) A="--eager";;
    graph1) A="";;
    *) A="--gshard-emulate ${v%b}";;
  esac
  timeout -k 10 300 $B $A > $O/m2.$v.json 2> $O/m2.$v.err
  rc=$?; echo "m2 $v rc=$rc $(summ $O/m2.$v.json)"; [ $rc -eq 0 ] || { tail -5 $O/m2.$v.err; exit $rc; }
done
