#!/bin/bash
# emit kernel time: in-tree lib vs ab/base.so, M5 kernel trace
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/emit_kt; mkdir -p $O
for v in base new; do
  if [ $v = base ]; then export GSPLAT_HIP_LIB=$GRAFT_REPO_ROOT/gsplat-triton_amd/ab/base.so; else unset GSPLAT_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$v -o k -- \
    /usr/bin/python3 bench.py --config m5 --no-cpu-baseline --no-traffic --steps 20 > $O/kt_$v.log 2>&1 || exit 2
  python -c "
import csv, glob
for f in glob.glob('$O/kt_$v/**/k_kernel_stats.csv', recursive=True) + glob.glob('$O/kt_$v/k_kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'st::' in r['Name'] or 'tight' in r['Name']: print('$v', r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
"
done
