"""One line per bench JSON under a gpurun_out/<tag> directory."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*.json")):
    try:
        d = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    r = d["roofline"]
    print(f"{f.split('/')[-1]:28s} {d['value']:8.1f} img/s  {d['ms_per_step']:.3f} ms/step  "
          f"fwd {r['launch_ms'] * 1e3:6.1f}  bwd {r['bwd']['launch_ms'] * 1e3:6.1f} us")
