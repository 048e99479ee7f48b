#!/bin/bash
# Rasterize-backward attribution (CFG=m2 default,
# CFG=m5 the 2DGS LEAN backward with the same bits): the bench's
# HIP-event backward time and the SQ wait counters of bwd2_kernel with parts
# of the per-record work switched off (GSPLAT_HIP_DBG, timing only):
#   0   full kernel          1   no atomics
#   5   no atomics, no cross-lane reduce-scatter
#   13  no atomics, no reduce-scatter, no gradient algebra (T recurrence,
#       exp / rcp, staging, culling, loads only)
#   (2DGS: +64 runs the attribution instance with nothing skipped, DBGS="0 64 65 69 77")
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-bwd_attr}; mkdir -p $O
CFG=${CFG:-m2}
for v in ${DBGS:-0 1 5 13}; do
  GSPLAT_HIP_DBG=$v timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-traffic --steps 20 \
    > $O/bench_dbg$v.json 2> $O/bench_dbg$v.err || exit 2
  python -c "import json; d=json.load(open('$O/bench_dbg$v.json')); print('dbg $v', round(d['value'],1), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
  GSPLAT_HIP_DBG=$v timeout -s KILL 120 rocprofv3 --kernel-include-regex "bwd2_kernel" \
    --pmc SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU \
    -f csv -d $O/pmc_dbg$v -o p -- /usr/bin/python3 bench.py --probe --config $CFG --warmup 2 > $O/pmc_dbg$v.log 2>&1 || exit 3
  GSPLAT_HIP_DBG=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "bwd2_kernel" -f csv \
    -d $O/kt_dbg$v -o k -- /usr/bin/python3 bench.py --probe --config $CFG --warmup 2 > $O/kt_dbg$v.log 2>&1 || exit 4
done
for v in ${DBGS:-0 1 5 13}; do echo "dbg $v"; python tools/pmc_summary.py $O/pmc_dbg$v; done > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
exit 0
