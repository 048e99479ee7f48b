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
