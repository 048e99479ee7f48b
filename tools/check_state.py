"""Compare the forward's chunk-boundary state (T, chunk colour sums) with the
float64 oracle rendering of the isect prefix (diagnostic)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import gsplat_hip
    from gsplat_hip import _lib
    from oracle import gsplat_oracle as O
    from test_gpu_parity import _garden_scene
    DEV = "cuda"
    L = 64
    C, N, W, H, D = 2, 12000, 100, 72, 3
    means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, seed=11, scale=0.12)
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
        means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
    tw, th = math.ceil(W / 16), math.ceil(H / 16)
    _, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th)
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    g = torch.Generator().manual_seed(5)
    cols = torch.rand(C, N, D, generator=g).to(DEV)
    ops = opac[None].repeat(C, 1).to(DEV)
    _lib.query("gsplat_hip_debug_set_chunk", L)
    ins = [x.detach().clone().requires_grad_(True) for x in (m2, cn, cols, ops)]
    rc, ra = gsplat_hip.rasterize_to_pixels(*ins, W, H, 16, off, fids)
    state = rc.grad_fn.saved_tensors[11].cpu().numpy()
    offs = off.reshape(-1).cpu().numpy().astype(np.int64)
    n = fids.numel()
    ends = np.append(offs[1:], n)
    fn = fids.cpu().numpy()
    args = [x.detach().cpu().numpy().astype(np.float64) for x in (m2, cn, cols, ops)]
    per = 256 * (1 + D)
    worst = []
    for t in np.argsort(-(ends - offs))[:6]:
        s0, e0 = offs[t], ends[t]
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        prev_acc = None
        for b in range(s0 + L, e0, L):
            # oracle: render the tile with its isect list cut at b (prefix)
            o2 = np.zeros_like(offs).reshape(C, th, tw)
            o2[...] = 0
            sub = fn[s0:b]
            o = np.full(C * th * tw, len(sub), np.int64)
            o[t] = 0
            with O.precision(np.float64):
                oc, oa, _ = O.raster_fwd(*args, None, W, H, 16, o.reshape(C, th, tw), sub)
            y0, x0 = ty * 16, tx * 16
            Tex = 1 - oa[c, y0:y0 + 16, x0:x0 + 16, 0]
            acc = oc[c, y0:y0 + 16, x0:x0 + 16]
            sl = state[(b // L) * per:(b // L + 1) * per]
            Tst = np.abs(sl[:256].reshape(16, 16))
            hh, ww = Tex.shape
            rel = np.abs(Tst[:hh, :ww] - Tex) / np.maximum(Tex, 1e-30)
            alive = Tex > 1e-3
            worst.append(float(rel[alive].max()) if alive.any() else 0.0)
            print(f"tile {t} n {e0 - s0} boundary {b - s0}: max rel T err (T>1e-3) "
                  f"{worst[-1]:.2e}  median {np.median(rel[alive]) if alive.any() else 0:.2e}")
    print("worst", max(worst))


if __name__ == "__main__":
    main()
