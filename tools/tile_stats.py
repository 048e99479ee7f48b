"""Tile-load statistics of one render of a bench config (isects per tile,
visible Gaussians, radii) -- run on the GPU box: python tools/tile_stats.py m5"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gsplat-triton_amd")]
import bench  # noqa: E402
from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "m2"
grid, W, H, _ = bench.CONFIGS[cfg]
means, rgbs, vms, Ks, sw, sh = load_garden_scene(os.path.join(ROOT, "tests/golden/garden_scene.npz"),
                                                 scene_grid=grid)
vm, K = camera_pool(vms, Ks, sw, sh, W, H, n=8)
tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", model=bench.MODEL.get(cfg, "3dgs"))
with torch.no_grad():
    _, _, meta = tr.render(0)
off = meta["isect_offsets"].flatten().long().cpu().numpy()
n = meta["flatten_ids"].numel()
cnt = np.diff(np.append(off, n))
r = meta["radii"].cpu().numpy().ravel()
tpg = meta["tiles_per_gauss"].cpu().numpy().ravel()
print(f"{cfg}: n_isects {n}, tiles {cnt.size}, per tile mean {cnt.mean():.0f} p50 {np.median(cnt):.0f} "
      f"p99 {np.percentile(cnt, 99):.0f} max {cnt.max()}")
print(f"visible {int((r > 0).sum())}, radii p50 {np.median(r[r > 0]):.0f} p99 {np.percentile(r[r > 0], 99):.0f} "
      f"max {r.max()}, tiles/gauss p99 {np.percentile(tpg[tpg > 0], 99):.0f} max {tpg.max()} "
      f"sum of top-100 {np.sort(tpg)[-100:].sum()}")
