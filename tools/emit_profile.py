"""Per-wave work of the supertile pair emission (csrc/isect_st.h emit_kernel)
at a bench config: the visible Gaussians in depth order (the emission's
order), their supertile counts np, and per wave of 64 the small-path rounds
(max np <= 16) and the big-path rounds (sum ceil(np / 64) over np > 16).

    python tools/emit_profile.py [m2|m5]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "m5"
    import bench
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene
    grid, W, H, _ = bench.CONFIGS[cfg]
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=grid)
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", model=bench.MODEL.get(cfg, "3dgs"))
    with torch.no_grad():
        _, _, meta = tr.render(0, 3)
    radii = meta["radii"][0]
    if radii.dim() > 1:
        radii = radii.amax(-1)
    m2 = meta["means2d"][0]
    d = meta["depths"][0]
    vis = radii > 0
    idx = torch.nonzero(vis).squeeze(1)
    idx = idx[torch.argsort(d[idx], stable=True)]
    r = radii[idx].float()
    p = m2[idx]
    ts = 16
    tw, th = (W + ts - 1) // ts, (H + ts - 1) // ts
    x0 = torch.clamp(torch.floor((p[:, 0] - r) / ts), 0, tw).int()
    x1 = torch.clamp(torch.ceil((p[:, 0] + r) / ts), 0, tw).int()
    y0 = torch.clamp(torch.floor((p[:, 1] - r) / ts), 0, th).int()
    y1 = torch.clamp(torch.ceil((p[:, 1] + r) / ts), 0, th).int()
    np_ = ((x1 - 1) // 4 - x0 // 4 + 1) * ((y1 - 1) // 4 - y0 // 4 + 1)
    np_ = torch.where((x1 > x0) & (y1 > y0), np_, torch.zeros_like(np_))
    n = np_.numel()
    pad = (-n) % 64
    w = torch.cat([np_, torch.zeros(pad, dtype=np_.dtype, device=np_.device)]).view(-1, 64)
    small = torch.where(w <= 16, w, torch.zeros_like(w)).amax(1)
    big = torch.where(w > 16, (w + 63) // 64, torch.zeros_like(w)).sum(1)
    print(f"{cfg}: visible {n}, pairs {int(np_.sum())}, big (>16) {int((np_ > 16).sum())} "
          f"holding {int(np_[np_ > 16].sum())} pairs")
    print("np quantiles", [int(x) for x in torch.quantile(np_.float(), torch.tensor(
        [0.5, 0.9, 0.99, 0.999, 1.0], device=np_.device))])
    print(f"waves {w.shape[0]}: small rounds mean {float(small.float().mean()):.2f} max "
          f"{int(small.max())}; big rounds mean {float(big.float().mean()):.2f} max "
          f"{int(big.max())}, waves with big rounds > 50: {int((big > 50).sum())}")
    top = torch.topk(big, 5)
    print("heaviest waves (index: big rounds)", list(zip(top.indices.tolist(), top.values.tolist())))


if __name__ == "__main__":
    main()
