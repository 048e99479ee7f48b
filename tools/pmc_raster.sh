#!/bin/bash
# SQ counters for the rasterizer kernels on the bench workload (two passes).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_raster}
mkdir -p $OUT
B="/usr/bin/python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-traffic"
timeout -k 10 300 rocprofv3 --kernel-include-regex r16 --pmc SQ_WAVES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_LDS -f csv -d $OUT/a -o p -- $B > $OUT/a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-include-regex r16 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d $OUT/b -o p -- $B > $OUT/b.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-include-regex r16 --pmc SQ_CYCLES SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM -f csv -d $OUT/c -o p -- $B > $OUT/c.log 2>&1 || exit 3
exit 0
