"""Host (Python) cost of the emulated 8-rank Gaussian-sharded M2 step
(bench.py --gshard-emulate 8): wall time per step, then cProfile over 20
steps, top functions by own time and by cumulative time."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)
from gsplat_hip import distributed as gdist  # noqa: E402
from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene  # noqa: E402

Wd = int(sys.argv[1]) if len(sys.argv) > 1 else 8
means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
    os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=3)
W, H = 1920, 1080
vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
gdist.EMULATION = gdist.Emulation(Wd)
for j in range(1, Wd):
    peer = Trainer(means, rgbs, vm, K, W, H, device="cuda", world_size=Wd, rank=j,
                   gaussian_shard=True, graph=False)
    gdist.EMULATION.record(j, lambda: peer.render(peer.camera_index(0)))
    del peer
tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", world_size=Wd, rank=0,
             gaussian_shard=True, graph=False)
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
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(40)
