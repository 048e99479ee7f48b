"""Print the kernels of the last full training step from a rocprofv3 kernel
trace (between the last two Adam launches): start offset, duration, name."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a + 1]["Start_Timestamp"])
busy = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f} {r['Kernel_Name'][:90]}")
end = int(rows[b]["End_Timestamp"])
print(f"step span {(end - t0) / 1000:.1f} us, kernel busy {busy / 1000:.1f} us")

# idle gaps over every full step in the trace: mean span / busy and the
# largest gaps with the kernels either side
gaps, spans, busys = {}, [], []
for a, b in zip(idx[:-1], idx[1:]):
    seg = rows[a + 1:b + 1]
    s0 = int(seg[0]["Start_Timestamp"])
    spans.append(int(seg[-1]["End_Timestamp"]) - int(rows[a]["End_Timestamp"]))
    busys.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg))
    prev = rows[a]
    for r in seg:
        g = int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])
        key = (prev["Kernel_Name"][:40], r["Kernel_Name"][:40])
        gaps.setdefault(key, []).append(g)
        prev = r
n = len(spans)
print(f"{n} steps: mean span {sum(spans) / n / 1000:.1f} us, mean busy {sum(busys) / n / 1000:.1f} us")
tot = sorted(((sum(v) / n, k) for k, v in gaps.items()), reverse=True)[:12]
for g, k in tot:
    print(f"  gap {g / 1000:7.1f} us/step  {k[0]}  ->  {k[1]}")
