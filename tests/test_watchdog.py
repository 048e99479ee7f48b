"""The progress watchdog (csrc/watchdog.cpp, distributed.Watchdog) on CPU.

A multi-GPU bench job must not die silently: when one rank never joins a
collective (bench.py --debug-hang RANK:STEP on the GPUs), every rank still
blocked ends with its rank, step and phase on stderr and a non-zero status
inside the timeout.  Here two gloo ranks stand in: rank 1 skips step 2's
all_reduce, so both ranks end up blocked in mismatched collectives (gloo's own
timeout is set far longer than the watchdog's), and both watchdogs fire.  A
second test checks the fallback text (the bench's main result line, still
delivered when a later phase hangs)."""

import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HANG = r"""
import datetime, os, sys, time
sys.path.insert(0, os.path.join(os.environ["ROOT"], "gsplat-triton_amd"))
import torch, torch.distributed as dist
from gsplat_hip.distributed import Watchdog
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", rank=rank, world_size=2,
                        timeout=datetime.timedelta(seconds=600))
wd = Watchdog(3.0, f"test rank {rank}/2")
wd.arm()
t = torch.ones(4)
for it in range(5):
    wd.beat(f"rank {rank} timed step {it}: replay")
    if rank == 1 and it == 2:
        continue  # this rank never joins step 2's collective
    dist.all_reduce(t)
wd.beat(f"rank {rank} final barrier")
dist.barrier()
print("finished", flush=True)
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_skipped_collective_ends_every_rank_with_a_diagnosis():
    port = _port()
    procs = []
    t0 = time.time()
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), WORLD_SIZE="2")
        procs.append(subprocess.Popen([sys.executable, "-c", HANG], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    elapsed = time.time() - t0
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        assert p.returncode == 3, (r, p.returncode, err[-2000:])
        assert "finished" not in out
        assert f"[gsplat_hip watchdog] test rank {r}/2: no progress for 3 s" in err, err[-2000:]
        assert f"last state: rank {r} " in err, err[-2000:]
    assert elapsed < 90, elapsed


FALLBACK = r"""
import os, sys, time
sys.path.insert(0, os.path.join(os.environ["ROOT"], "gsplat-triton_amd"))
from gsplat_hip.distributed import Watchdog
wd = Watchdog(1.0, "test")
wd.arm("phase 2")
wd.fallback(1, '{"value": 1.0, "dp": "hung"}\n', 0)
time.sleep(60)
print("not reached", flush=True)
"""


def test_fallback_line_is_delivered_on_expiry():
    p = subprocess.run([sys.executable, "-c", FALLBACK], env=dict(os.environ, ROOT=ROOT),
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout == '{"value": 1.0, "dp": "hung"}\n', p.stdout
    assert "last state: phase 2" in p.stderr


DISARM = r"""
import os, sys, time
sys.path.insert(0, os.path.join(os.environ["ROOT"], "gsplat-triton_amd"))
from gsplat_hip.distributed import Watchdog
wd = Watchdog(0.5, "test")
wd.arm()
for i in range(6):
    time.sleep(0.2)
    wd.beat(f"step {i}")
wd.disarm()
time.sleep(1.5)
print("ok", flush=True)
"""


def test_beats_and_disarm_keep_the_process_alive():
    p = subprocess.run([sys.executable, "-c", DISARM], env=dict(os.environ, ROOT=ROOT),
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and p.stdout == "ok\n", (p.returncode, p.stderr[-2000:])
