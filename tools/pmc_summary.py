"""Summarise rocprofv3 --pmc CSVs (tools/pmc_kernels.sh output): mean counter
value per kernel name over all dispatches, one column per counter."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/*/p_counter_collection.csv") + glob.glob(f"{root}/p_counter_collection.csv"):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (d, c), v in per.items():
        vals[names[d][:60]][c].append(v)
for k, cs in sorted(vals.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.4g}")
