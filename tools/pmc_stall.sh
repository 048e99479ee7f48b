#!/bin/bash
# Stall breakdown of the rasterizer kernels on the M2 bench workload: one
# rocprofv3 --pmc pass per counter group (SQ <= 8, TCP <= 4, TCC <= 4 per pass),
# each under its own time limit; summary per kernel in $O/summary.txt.
# usage: tools/pmc_stall.sh TAG [kernel regex]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-stall}
R=${2:-'r16::(fwd|bwd2)_kernel'}
O=gpurun_out/$TAG; mkdir -p $O
B="/usr/bin/python3 bench.py --probe --warmup 2"
i=0
while read -r CTRS; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$R" --pmc $CTRS -f csv -d $O/p$i -o p -- $B \
    > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc: $CTRS"; [ $rc -eq 0 ] || exit $rc
done <<'EOF'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_LEVEL_WAVES
EOF
python tools/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
