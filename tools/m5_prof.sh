cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/m5_bench.sh r6_x/m5 || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r6_x/pmc
mkdir -p $OUT
B="/usr/bin/python3 bench.py --config m5 --steps 3 --warmup 2 --no-cpu-baseline --no-traffic"
timeout -k 10 300 rocprofv3 --kernel-include-regex "surfel::(bwd2|fwd2s)" -f csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $OUT/a -o p -- $B > $OUT/a.log 2>&1 || exit 2
python tools/pmc_summary.py $OUT
