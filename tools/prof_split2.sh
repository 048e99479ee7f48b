#!/bin/bash
# Kernel statistics of the M2 / M3 step per split setting (GSPLAT_HIP_FWD_SPLIT_DIV
# or off), eager steps.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-prof_split2}; mkdir -p $O
for cfg in ${PS_CFGS:-m2}; do
  for v in ${PS_VARS:-off 550 2000}; do
    unset GSPLAT_HIP_FWD_SPLIT GSPLAT_HIP_FWD_SPLIT_DIV
    if [ $v = off ]; then export GSPLAT_HIP_FWD_SPLIT=0; else export GSPLAT_HIP_FWD_SPLIT_DIV=$v; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/$cfg.$v -o run -- /usr/bin/python3 bench.py --steps 10 --warmup 3 --eager --no-cpu-baseline --no-traffic --config $cfg > $O/$cfg.$v.log 2>&1 || exit 1
    echo "$cfg $v done"
  done
done
