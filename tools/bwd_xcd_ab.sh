#!/bin/bash
# XCD-aware backward item order: L2 counters of the 3DGS backward at M2 and
# M3 for the in-tree library against gsplat-triton_amd/ab/base.so, then M3
# bench lines alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-bwd_xcd}; mkdir -p $O
for cfg in m2 m3; do
  for v in base new; do
    if [ $v = base ]; then export GSPLAT_HIP_LIB=$GRAFT_REPO_ROOT/gsplat-triton_amd/ab/base.so; else unset GSPLAT_HIP_LIB; fi
    for ctr in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
      tag=$(echo $ctr | cut -c1-5)
      timeout -s KILL 150 rocprofv3 --kernel-include-regex "r16::bwd2_kernel" --pmc $ctr -f csv \
        -d $O/pmc_${cfg}_${v}_$tag -o p -- /usr/bin/python3 bench.py --config $cfg --probe --warmup 2 \
        > $O/pmc_${cfg}_${v}_$tag.log 2>&1 || exit 3
    done
    python - <<PY
import csv, collections, glob
per = collections.defaultdict(float)
for f in glob.glob("$O/pmc_${cfg}_${v}_*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        per[(f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
c = collections.defaultdict(list)
for (f, d, k), x in per.items(): c[k].append(x)
m = {k: sum(x) / len(x) for k, x in c.items()}
hit = m.get("TCC_HIT_sum", 0); miss = m.get("TCC_MISS_sum", 0)
print("$cfg $v bwd2", "l2_hit", round(hit / max(hit + miss, 1), 3), "fetch_MB x2", round(2 * m.get("FETCH_SIZE", 0) / 1024, 1))
PY
  done
done
unset GSPLAT_HIP_LIB
CFG=m3 bash tools/ab_lib.sh ${1:-bwd_xcd}/m3
exit 0
