#!/bin/bash
# One GPU-box session: the -m gpu suite (up to 10 failures reported), an M2
# bench line and a one-GPU line with the data-parallel phase (the N>1 code
# path on a 1-rank RCCL group).  Each GPU step has its own time limit; after a
# crash / abort / time limit nothing else runs.
# usage: tools/run_suite.sh TAG [pytest selection...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; shift; mkdir -p $O
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -q --maxfail=10 --timeout 200 \
  --timeout-method thread > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 $O/suite.log | grep -E "passed|failed|FAILED|Error" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic > $O/bench_m2.json 2> $O/bench_m2.err
r2=$?; echo "bench m2 rc=$r2"; [ $r2 -eq 0 ] || exit $r2
python -c "import json; d=json.load(open('$O/bench_m2.json')); print('m2', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', d['roofline']['launch_ms'], 'bwd', d['roofline']['bwd']['launch_ms'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --dp-phase > $O/bench_dpphase.json 2> $O/bench_dpphase.err
r3=$?; echo "bench dp-phase rc=$r3"; [ $r3 -eq 0 ] || exit $r3
python -c "import json; d=json.load(open('$O/bench_dpphase.json')); print('m2', round(d['value'],1), 'dp', d['config'].get('dp'))"
exit $rc
