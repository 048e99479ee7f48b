"""Per-step kernel timeline of a rocprofv3 kernel trace: finds the graph-
replayed training steps (from one activate_fwd_fetch launch to the next),
and reports the GPU-busy time, the idle gaps between consecutive kernels and
the span per step.  usage: python tools/step_gaps.py run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "activate_fwd_kernel<true>" in r["Kernel_Name"]]
spans, busy, gaps, nk = [], [], [], []
for a, b in zip(starts, starts[1:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    bsy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gp = sum(max(0, int(seg[i + 1]["Start_Timestamp"]) - int(seg[i]["End_Timestamp"]))
             for i in range(len(seg) - 1))
    spans.append(t1 - t0)
    busy.append(bsy)
    gaps.append(gp)
    nk.append(len(seg))
# the timed, graph-replayed steps: the run of equal-length segments with the
# most kernels is the training step
if not spans:
    sys.exit("no steps found")
med = sorted(spans)[len(spans) // 2]
print(f"steps {len(spans)}; median span {med / 1e3:.1f} us")
for s, b_, g, k in zip(spans, busy, gaps, nk):
    print(f"span {s / 1e3:8.1f} us  busy {b_ / 1e3:8.1f}  gaps {g / 1e3:7.1f}  kernels {k}")
