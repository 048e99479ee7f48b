#!/bin/bash
# Fused SSIM blocking variants (GSPLAT_HIP_SSIM_FV 0-7, csrc/ssim.hip):
# parity tests per variant, loss fwd+bwd microbench with a fingerprint of the
# loss and gradient (re-blocked variants must agree bit for bit), kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${AB_TAG:-ssim3}; mkdir -p $O
for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
  GSPLAT_HIP_SSIM_FV=$v timeout -k 10 200 python -u -m pytest tests/test_gpu_trainer.py -x -q -k "l1_ssim_loss or fused_loss" --timeout 120 --timeout-method thread > $O/tests_v$v.log 2>&1 || { tail -30 $O/tests_v$v.log; exit 1; }
  echo "v$v: $(tail -1 $O/tests_v$v.log)"
done
timeout -k 10 120 python -u tools/ssim_bench.py 0 >> $O/micro.txt 2>&1 || exit 2
for rep in 1 2; do
  for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
    GSPLAT_HIP_SSIM_FV=$v timeout -k 10 120 python -u tools/ssim_bench.py 1 >> $O/micro.txt 2>&1 || exit 3
  done
done
for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
  GSPLAT_HIP_SSIM_FV=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/v$v -o run -- /usr/bin/python3 tools/ssim_bench.py 1 > /dev/null 2>&1 || exit 4
done
cat $O/micro.txt
python3 - "$O" <<'PY'
import csv, glob, re, sys
for f in sorted(glob.glob(sys.argv[1] + "/v*/**/*kernel_stats.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "fused_kernel" in r["Name"]:
            print(re.search(r"/(v\d)/", f).group(1), r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
exit 0
