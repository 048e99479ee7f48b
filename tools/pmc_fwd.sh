# One PMC pass (issue/stall counters) over the rasterizer kernels of the bench workload.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${PMC_TAG:-pmcf}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-include-regex "r16" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY -f csv -d $O/p1 -o p -- /usr/bin/python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-traffic > $O/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-include-regex "r16" --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d $O/p2 -o p -- /usr/bin/python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-traffic > $O/p2.log 2>&1 || exit 2
python tools/pmc_summary.py $O > $O/summary.txt
