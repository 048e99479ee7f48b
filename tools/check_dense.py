"""Dense-scene accuracy of the rasterizer backward against the float64 oracle
(diagnostic; prints bad-row counts at the reference tolerances)."""
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
    from test_gpu_parity import _garden_scene, _last_ids
    DEV = "cuda"
    for seed, scale, N in ((11, 0.12, 12000), (3, 0.05, 4000)):
        C, W, H, D = 2, 100, 72, 3
        means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, seed=seed, scale=scale)
        radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
            means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
        tw, th = math.ceil(W / 16), math.ceil(H / 16)
        _, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th)
        off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
        g = torch.Generator().manual_seed(5)
        cols = torch.rand(C, N, D, generator=g).to(DEV)
        ops = opac[None].repeat(C, 1).to(DEV)
        bg = torch.rand(C, D, generator=g).to(DEV)
        vrc = torch.randn(C, H, W, D, generator=g).to(DEV)
        vra = torch.randn(C, H, W, 1, generator=g).to(DEV)
        for L in (0, 64):
            _lib.query("gsplat_hip_debug_set_chunk", L)
            ins = [x.detach().clone().requires_grad_(True) for x in (m2, cn, cols, ops)]
            rc, ra = gsplat_hip.rasterize_to_pixels(*ins, W, H, 16, off, fids, backgrounds=bg)
            grads = torch.autograd.grad((rc * vrc).sum() + (ra * vra).sum(), ins,
                                        retain_graph=True)
            args = [x.detach().cpu().numpy().astype(np.float64) for x in (m2, cn, cols, ops, bg)]
            for prec in (np.float32, np.float64):
                with O.precision(prec):
                    ref = O.raster_bwd(*args, W, H, 16, off.cpu().numpy(), fids.cpu().numpy(),
                                       ra.detach().cpu().numpy().astype(prec), _last_ids(rc),
                                       vrc.cpu().numpy().astype(prec),
                                       vra.cpu().numpy().astype(prec))
                out = []
                for k, (tol, nm) in enumerate(((5e-3, "mean"), (1e-3, "conic"), (1e-3, "color"),
                                               (2e-3, "opac"))):
                    a = grads[k].detach().cpu().numpy().astype(np.float64)
                    b = np.asarray(ref[k], np.float64)
                    bad = ~np.isclose(a, b, rtol=tol, atol=tol)
                    if bad.ndim > 1 and a.shape[-1] > 1:
                        bad = bad.reshape(-1, a.shape[-1]).any(-1)
                    out.append(f"{nm} {bad.sum()} ({np.abs(a - b).max():.2e})")
                print(f"seed {seed} N {N} chunk {L} vs {np.dtype(prec).name}: " + ", ".join(out))
        _lib.query("gsplat_hip_debug_set_chunk", 1024)


if __name__ == "__main__":
    main()
