#!/bin/bash
# A/B of two builds of the library on one box, alternating: the in-tree
# library ("new") against gsplat-triton_amd/ab/base.so ("base"), bench lines
# of config $CFG (default m5).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_lib}; mkdir -p $O
CFG=${CFG:-m5}
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export GSPLAT_HIP_LIB=$GRAFT_REPO_ROOT/gsplat-triton_amd/ab/base.so; else unset GSPLAT_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-traffic --steps 30 \
      > $O/bench_${CFG}_${v}_$r.json 2> $O/bench_${CFG}_${v}_$r.err || exit 2
    python -c "import json; d=json.load(open('$O/bench_${CFG}_${v}_$r.json')); print('$CFG $v run $r', round(d['value'],1), round(d['ms_per_step'],4), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  done
done
exit 0
