"""Host timeline of one M2 training step: wall-clock time (us) of every
C-ABI call relative to the step start, to see where the host lags the GPU
(e.g. after the n_isects sync)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)

from gsplat_hip import _lib  # noqa: E402
from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene  # noqa: E402

means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
    os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=3)
W, H = 1920, 1080
vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
tr = Trainer(means, rgbs, vm, K, W, H, device="cuda")
for it in range(5):
    tr.step(it)
torch.cuda.synchronize()
log = []
orig_call = _lib.call


def call(name, *args):
    t = time.perf_counter()
    r = orig_call(name, *args)
    log.append((t, time.perf_counter(), name))
    return r


_lib.call = call
orig_item = torch.Tensor.item
for it in range(3):
    log.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.step(it)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"step {it}: host {1e6 * (t1 - t0):.0f} us")
for a, b, n in log:
    print(f"{1e6 * (a - t0):8.1f} {1e6 * (b - a):7.1f}  {n}")
