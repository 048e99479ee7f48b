"""Summarise a rocprofv3 kernel_stats.csv: per-step microseconds by kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e3 / steps:.1f} us per step ({steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{int(r['Calls']):>6} {float(r['AverageNs']) / 1e3:8.1f}us {float(r['TotalDurationNs']) / 1e3 / steps:8.1f}us/step "
          f"{float(r['Percentage']):6.2f}% {r['Name'][:100]}")
