"""Host (Python) cost of the M2 training step: cProfile over 20 steps, top
functions by own time."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)
from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene  # noqa: E402

means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
    os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=3)
W, H = 1920, 1080
vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
tr = Trainer(means, rgbs, vm, K, W, H, device="cuda")
for it in range(5):
    tr.step(it)
torch.cuda.synchronize()
t0 = time.perf_counter()
for it in range(5, 25):
    tr.step(it)
torch.cuda.synchronize()
print(f"wall per step {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
for it in range(25, 45):
    tr.step(it)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
