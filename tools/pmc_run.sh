#!/bin/bash
# PMC passes on the bench workload, rasterizer + main kernels only.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${PMC_TAG:-pmc8}
mkdir -p $OUT
B="/usr/bin/python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-traffic"
R='r16|adam|sh_bwd|ssim'
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -f csv -d $OUT/p1 -o p -- $B > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc FETCH_SIZE -f csv -d $OUT/p2 -o p -- $B > $OUT/p2.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc WRITE_SIZE -f csv -d $OUT/p3 -o p -- $B > $OUT/p3.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-include-regex "$R" --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD -f csv -d $OUT/p4 -o p -- $B > $OUT/p4.log 2>&1 || echo "p4 failed"
exit 0
