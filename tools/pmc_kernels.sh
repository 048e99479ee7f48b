#!/bin/bash
# SQ + memory counters for the kernels matching $2 on the bench workload.
# usage: tools/pmc_kernels.sh <outdir-name> <kernel-regex>
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_k}
R=${2:-ssim}
mkdir -p $OUT
B="/usr/bin/python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-traffic"
P="rocprofv3 --kernel-include-regex $R -f csv"
timeout -k 10 300 $P --pmc SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $OUT/a -o p -- $B > $OUT/a.log 2>&1 || exit 1
timeout -k 10 300 $P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES -d $OUT/b -o p -- $B > $OUT/b.log 2>&1 || exit 2
timeout -k 10 300 $P --pmc FETCH_SIZE -d $OUT/c -o p -- $B > $OUT/c.log 2>&1 || exit 3
timeout -k 10 300 $P --pmc WRITE_SIZE -d $OUT/d -o p -- $B > $OUT/d.log 2>&1 || exit 4
exit 0
