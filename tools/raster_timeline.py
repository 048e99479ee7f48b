"""Per-wave timeline of the 16x16 rasterizer kernels on the bench workload.

    python tools/raster_timeline.py [--config m2] [--cam 0] [--out gpurun_out/tl.npz]

Runs a few training steps of bench.py's workload, then one render + backward
with gsplat_hip_debug_set_timeline() enabled, and reports for the forward and
the backward kernel: span, mean concurrency, when 50/90/99 % of the waves had
finished, and the slowest waves with their tile's isect count and its
effective length (isects up to the tile's largest last_id).  A profiling aid,
not part of the product path.
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def summarize(name, tl, n_isect_tile, n_eff_tile, per_tile=True):
    st, en = tl[:, 0].astype(np.int64), tl[:, 1].astype(np.int64)
    ok = en > 0
    t0 = st[ok].min()
    st, en = (st - t0) * 0.01, (en - t0) * 0.01  # 100 MHz ticks -> us
    dur = en - st
    span = en[ok].max()
    print(f"== {name}: span {span:.1f} us, waves {ok.sum()}, mean wave {dur[ok].mean():.2f} us, "
          f"max wave {dur[ok].max():.1f} us, mean concurrency {dur[ok].sum() / span:.0f}")
    ends = np.sort(en[ok])
    for q in (0.5, 0.9, 0.99, 0.999):
        print(f"   {q * 100:5.1f}% of waves done at {ends[int(q * (len(ends) - 1))]:.1f} us")
    # concurrency profile in 20 buckets
    edges = np.linspace(0, span, 21)
    conc = [((st[ok] < b) & (en[ok] > a)).sum() for a, b in zip(edges[:-1], edges[1:])]
    print("   active waves per 5% of span:", conc)
    if not per_tile:  # chunked backward: waves are (tile, chunk) work items
        print(f"   slowest waves (us): {np.round(np.sort(dur[ok])[-8:], 1).tolist()}")
        return
    tiles = np.arange(len(tl)) // 4
    order = np.argsort(-dur)
    print("   slowest waves: (us, start, tile, isects, n_eff)")
    for w in order[:12]:
        t = tiles[w]
        print(f"     {dur[w]:7.1f} {st[w]:7.1f} {t:6d} {n_isect_tile[t]:6d} {n_eff_tile[t]:6d}")
    # correlation of wave time with per-tile work
    tt = np.zeros(len(n_isect_tile))
    np.maximum.at(tt, tiles[ok], dur[ok])
    print(f"   per-tile time vs n_eff: corr {np.corrcoef(tt, n_eff_tile)[0, 1]:.3f}; "
          f"us per 1k n_eff (heaviest 1%): "
          f"{np.median(tt[n_eff_tile >= np.quantile(n_eff_tile, 0.99)] / np.maximum(n_eff_tile[n_eff_tile >= np.quantile(n_eff_tile, 0.99)], 1) * 1000):.2f}")


def meta_isects_bound(tr, cam):
    """Upper bound on the chunked backward's work items / 4 (waves)."""
    with torch.no_grad():
        _, _, meta = tr.render(cam)
    return meta["isect_ids"].numel() // 64 + 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="m2")
    ap.add_argument("--cam", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import bench
    from gsplat_hip import _lib
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene

    grid, W, H, _ = bench.CONFIGS[args.config]
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=grid)
    vm_pool, K_pool = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device="cuda")
    for it in range(3):
        tr.step(it)
    torch.cuda.synchronize()

    tw, th = (W + 15) // 16, (H + 15) // 16
    n_tiles = tw * th
    buf_f = torch.zeros(4 * n_tiles * 2, dtype=torch.int64, device="cuda")
    buf_b = torch.zeros(4 * (2 * n_tiles + meta_isects_bound(tr, args.cam)) * 2,
                        dtype=torch.int64, device="cuda")
    _lib.call("gsplat_hip_debug_set_timeline", buf_f.data_ptr(), 4 * n_tiles)
    colors, alphas, meta = tr.render(args.cam)
    torch.cuda.synchronize()
    last = None
    for t in colors.grad_fn.saved_tensors:
        if t is not None and t.dtype == torch.int32 and t.dim() == 3 and t.shape[1:] == (H, W):
            last = t.clone()
    _lib.call("gsplat_hip_debug_set_timeline", buf_b.data_ptr(), buf_b.numel() // 2)
    from gsplat_hip.losses import l1_ssim_loss
    loss = l1_ssim_loss(colors, tr.targets[args.cam:args.cam + 1], 0.2)
    loss.backward()
    torch.cuda.synchronize()
    _lib.call("gsplat_hip_debug_set_timeline", 0, 0)

    off = meta["isect_offsets"].reshape(-1).long().cpu().numpy()
    n_is = meta["isect_ids"].numel()
    ends = np.append(off[1:], n_is)
    n_isect_tile = ends - off
    # effective length: isects up to the largest last_id in the tile
    if last is None:
        n_eff = n_isect_tile
    else:
        lt = last[0].cpu().numpy()
        pad = np.zeros((th * 16, tw * 16), np.int64) - 1
        pad[:H, :W] = lt
        mx = pad.reshape(th, 16, tw, 16).max(axis=(1, 3)).reshape(-1)
        n_eff = np.clip(np.minimum(ends, mx + 1) - off, 0, None)
    print(f"tiles {n_tiles}, isects {n_is}, per-tile isects mean {n_isect_tile.mean():.0f} "
          f"max {n_isect_tile.max()}, n_eff mean {n_eff.mean():.0f} max {n_eff.max()} "
          f"sum {n_eff.sum()}")
    tf = buf_f.view(-1, 2).cpu().numpy().view(np.uint64)
    tb = buf_b.view(-1, 2).cpu().numpy().view(np.uint64)
    summarize("rasterize fwd", tf, n_isect_tile, n_eff)
    summarize("rasterize bwd", tb, n_isect_tile, n_eff, per_tile=len(tb) == 4 * n_tiles)
    if args.out:
        np.savez_compressed(args.out, fwd=tf, bwd=tb, n_isect_tile=n_isect_tile, n_eff=n_eff)


if __name__ == "__main__":
    main()
