"""Dump one render's projected visible Gaussians (means2d, radii, depths) of a
bench config for CPU-side isect studies -- run on the GPU box:
    python tools/isect_dump.py m2 gpurun_out/isect_m2.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gsplat-triton_amd")]
import bench  # noqa: E402
from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "m2"
out = sys.argv[2] if len(sys.argv) > 2 else f"gpurun_out/isect_{cfg}.npz"
grid, W, H, _ = bench.CONFIGS[cfg]
means, rgbs, vms, Ks, sw, sh = load_garden_scene(os.path.join(ROOT, "tests/golden/garden_scene.npz"),
                                                 scene_grid=grid)
vm, K = camera_pool(vms, Ks, sw, sh, W, H, n=8)
tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", model=bench.MODEL.get(cfg, "3dgs"),
             graph=False)
with torch.no_grad():
    _, _, meta = tr.render(0)
r = meta["radii"].flatten()
vis = torch.nonzero(r > 0).flatten()
np.savez_compressed(out, W=W, H=H, idx=vis.int().cpu().numpy(),
                    radii=r[vis].cpu().numpy(),
                    means2d=meta["means2d"].reshape(-1, 2)[vis].cpu().numpy(),
                    depths=meta["depths"].flatten()[vis].cpu().numpy(),
                    n_isects=meta["flatten_ids"].numel())
print(cfg, "visible", vis.numel(), "isects", meta["flatten_ids"].numel())
