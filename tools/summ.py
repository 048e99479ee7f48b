"""Print a bench line's headline numbers and the top kernels of a rocprofv3 stats CSV."""
import csv
import json
import sys

d = sys.argv[1]
try:
    b = json.load(open(f"{d}/bench.json"))
    r = b["roofline"]
    print(f"value {b['value']:.1f} {b['unit']}  ms/step {b['ms_per_step']:.3f}  "
          f"fwd {r['launch_ms']:.3f} ms  bwd {r['rasterize_bwd_ms']:.3f} ms  frac {r['frac']:.4f}")
except Exception as e:  # noqa: BLE001
    print("no bench line:", e)
rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f}us "
          f"{float(r['Percentage']):6.2f}%")
