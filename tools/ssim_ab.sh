#!/bin/bash
# SSIM+L1 fused loss: kernel time of the in-tree library against
# gsplat-triton_amd/ab/base.so (rocprofv3 kernel trace of tools/ssim_bench.py
# at 1080p RGB), alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ssim_ab}; mkdir -p $O
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export GSPLAT_HIP_LIB=$GRAFT_REPO_ROOT/gsplat-triton_amd/ab/base.so; else unset GSPLAT_HIP_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_${v}_$r -o k -- \
      /usr/bin/python3 tools/ssim_bench.py 1 > $O/kt_${v}_$r.log 2>&1 || exit 2
    python -c "
import csv, glob
for f in glob.glob('$O/kt_${v}_$r/**/k_kernel_stats.csv', recursive=True) + glob.glob('$O/kt_${v}_$r/k_kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'ssim' in r['Name']: print('$v $r', r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
"
  done
done
exit 0
