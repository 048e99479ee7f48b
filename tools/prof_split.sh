# rocprofv3 kernel stats of the M2 bench with the split forward on / off.
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${PS_TAG:-profsplit}; mkdir -p $O
for sp in -1 0; do
  GSPLAT_HIP_FWD_SPLIT=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/s$sp -o run -- /usr/bin/python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --config ${PS_CFG:-m2} > $O/s$sp.log 2>&1 || exit 1
done
