# Split-forward threshold A/B on M2 / M3: off, a threshold above every tile,
# and adaptive thresholds n_isects / DIV.
set -o pipefail
O=gpurun_out/${AB_TAG:-absd}; mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-traffic"
for cfg in ${AB_CFGS:-m2 m3}; do
  for v in ${AB_V:-off big d550 d400 off big d550 d400}; do
    sp=-1; dv=640
    case $v in off) sp=0;; big) sp=100000;; d*) dv=${v#d};; esac
    GSPLAT_HIP_FWD_SPLIT=$sp GSPLAT_HIP_FWD_SPLIT_DIV=$dv GSPLAT_HIP_FWD_SPLIT_CHUNK=512 timeout -k 10 200 $B --config $cfg > $O/$cfg.$v.$RANDOM.json 2>>$O/err.log || exit 2
  done
done
