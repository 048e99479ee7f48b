#!/bin/bash
# A/B of the XCD-grouped forward dispatch order (GSPLAT_HIP_DBG=16) at M2 and
# M3 with L2 counters: bench lines (HIP-event launch times) alternating, then
# TCC hit / miss and FETCH_SIZE of the forward per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-xcd_ab}; mkdir -p $O
# M3: the split forward on (the default), off, off + grouped order, and off
# with no chunk-state stores (traffic attribution)
for cfg in m2 m3; do
  if [ $cfg = m3 ]; then VARS="s 0 16 32"; else VARS="0 16"; fi
  for r in 1 2; do
    for v in $VARS; do
      if [ $v = s ]; then SPL=""; DB=0; else SPL=0; DB=$v; fi
      [ $cfg = m2 ] && SPL=""
      GSPLAT_HIP_FWD_SPLIT=$SPL GSPLAT_HIP_DBG=$DB timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-traffic --steps 20 \
        > $O/bench_${cfg}_dbg${v}_$r.json 2> $O/bench_${cfg}_dbg${v}_$r.err || exit 2
      python -c "import json; d=json.load(open('$O/bench_${cfg}_dbg${v}_$r.json')); print('$cfg dbg $v run $r', round(d['value'],1), 'fwd', round(d['roofline']['launch_ms'],4), 'bwd', round(d['roofline']['bwd']['launch_ms'],4))"
    done
  done
  for v in $VARS; do
    if [ $v = s ]; then SPL=""; DB=0; else SPL=0; DB=$v; fi
    [ $cfg = m2 ] && SPL=""
    for ctr in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
      tag=$(echo $ctr | cut -c1-5)
      GSPLAT_HIP_FWD_SPLIT=$SPL GSPLAT_HIP_DBG=$DB timeout -s KILL 150 rocprofv3 --kernel-include-regex "fwd_kernel" --pmc $ctr \
        -f csv -d $O/pmc_${cfg}_dbg${v}_$tag -o p -- /usr/bin/python3 bench.py --config $cfg --probe --warmup 2 \
        > $O/pmc_${cfg}_dbg${v}_$tag.log 2>&1 || exit 3
    done
    python - <<PY
import csv, collections, glob
per = collections.defaultdict(float)
for f in glob.glob("$O/pmc_${cfg}_dbg${v}_*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        per[(f, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
c = collections.defaultdict(list)
for (f, d, k), x in per.items(): c[k].append(x)
m = {k: sum(x) / len(x) for k, x in c.items()}
hit = m.get("TCC_HIT_sum", 0); miss = m.get("TCC_MISS_sum", 0)
print("$cfg dbg $v", {k: "%.4g" % x for k, x in m.items()}, "l2_hit", round(hit / max(hit + miss, 1), 3), "fetch_MB x2", round(2 * m.get("FETCH_SIZE", 0) / 1024, 1))
PY
  done
done
exit 0
