#!/bin/bash
# Round-4 batch 10: SH Adam rows non-temporal (GSPLAT_HIP_SH_ADAM_NT) A/B at
# M2, alternating, with a kernel trace of each; SH tests under NT=1; then
# batch 11 (the trainer-chosen split divisor) in the same call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_batch10}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print(round(d['value'],1), round(d['ms_per_step'],3), 'fwd', round(r['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4))"; }
GSPLAT_HIP_SH_ADAM_NT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_trainer.py -q -k "sh or graph or adam" --timeout 180 --timeout-method thread > $O/tests_nt.log 2>&1
rc=$?; echo "tests (NT=1) rc=$rc"; grep FAILED $O/tests_nt.log; tail -1 $O/tests_nt.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for nt in 0 1; do
    GSPLAT_HIP_SH_ADAM_NT=$nt timeout -k 10 300 python -u bench.py --no-traffic --no-cpu-baseline > $O/m2_nt$nt.$r.json 2> $O/m2_nt$nt.$r.err || exit 2
    echo "m2 nt=$nt run $r $(v $O/m2_nt$nt.$r.json)"
  done
done
for nt in 0 1; do
  GSPLAT_HIP_SH_ADAM_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_nt$nt -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $O/trace_nt$nt.log 2>&1 || exit 6
done
python3 - $O <<'PY'
import csv, glob, sys
for nt in (0, 1):
    for f in glob.glob(sys.argv[1] + f"/trace_nt{nt}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any(k in r["Name"] for k in ("sh_bwd", "adam::step", "bwd2_kernel", "fwd_kernel<3, 0, false>", "fused_kernel")):
                print(f"nt={nt}", r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
tools/r4_batch11.sh ${1:-r4_batch10}/b11 || exit 7
