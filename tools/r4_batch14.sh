#!/bin/bash
# Round-4 batch 14: SH backward without per-lane 64-bit division (the camera
# and row are known): GPU suite, M2 twice, kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch14}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep FAILED $O/tests.log; tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2.$r.json 2> $O/m2.$r.err || exit 2
  echo "m2 run $r $(v $O/m2.$r.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace.log 2>&1 || exit 6
python3 - $O <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("sh_fwd", "sh_bwd", "bwd2_kernel")):
            print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
