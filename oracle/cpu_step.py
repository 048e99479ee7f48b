"""CPU baseline for bench.py: one training step of the hot path computed by
the numpy oracle (test infrastructure; only bench.py's cpu_baseline leg and
tests use it).

Bounded sample: projection, SH, isect (+sort, offsets), the loss gradient and
Adam run on the full workload; rasterize forward/backward run on every
`tile_stride`-th tile and are scaled by the number of tiles to estimate the
full-image time.  Single-threaded numpy (cores = 1).
"""

import math
import time

import numpy as np

from . import gsplat_oracle as O


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def cpu_train_step(means, quats, log_scales, logit_opac, sh, viewmat, K, width, height,
                   target, tile_stride=16, sh_degree=3, tile_size=16):
    """Returns (seconds_estimate_for_full_step, breakdown dict, sample description)."""
    t = {}
    f32 = np.float32
    C = 1
    t0 = time.perf_counter()
    scales = np.exp(log_scales).astype(f32)
    opac = _sigmoid(logit_opac).astype(f32)
    radii, m2, d, cn, _ = O.proj_fwd(means, quats, scales, viewmat[None], K[None], width, height)
    t["proj_fwd"] = time.perf_counter() - t0

    t0 = time.perf_counter()
    c2w = np.linalg.inv(viewmat)
    dirs = (means - c2w[:3, 3])[None].astype(f32)
    masks = radii > 0
    colors = O.sh_fwd(sh_degree, dirs, sh[None], masks)
    colors = np.maximum(colors + f32(0.5), 0).astype(f32)
    t["sh_fwd"] = time.perf_counter() - t0

    t0 = time.perf_counter()
    tw, th = math.ceil(width / tile_size), math.ceil(height / tile_size)
    _, ids, fids = O.isect_tiles(m2, radii, d, tile_size, tw, th)
    off = O.isect_offset_encode(ids, C, tw, th)
    t["isect"] = time.perf_counter() - t0

    n_tiles = C * tw * th
    tiles = list(range(0, n_tiles, tile_stride))
    scale = n_tiles / len(tiles)
    ops = opac[None]
    t0 = time.perf_counter()
    rc, ra, last = O.raster_fwd(m2, cn, colors, ops, None, width, height, tile_size, off, fids,
                                tiles=tiles)
    t["raster_fwd"] = (time.perf_counter() - t0) * scale

    t0 = time.perf_counter()
    # L1 part of the loss gradient (the SSIM part costs the same order; glue)
    v_rc = (np.sign(rc - target[None]) * (0.8 / rc.size)).astype(f32)
    v_ra = np.zeros_like(ra)
    t["loss"] = time.perf_counter() - t0

    t0 = time.perf_counter()
    vm2, vcn, vcol, vop, _, _ = O.raster_bwd(m2, cn, colors, ops, None, width, height, tile_size,
                                             off, fids, ra, last, v_rc, v_ra, tiles=tiles)
    t["raster_bwd"] = (time.perf_counter() - t0) * scale

    t0 = time.perf_counter()
    v_sh, v_dirs = O.sh_bwd(sh_degree, dirs, sh[None], vcol * (colors > 0), masks, True)
    t["sh_bwd"] = time.perf_counter() - t0

    t0 = time.perf_counter()
    O.proj_bwd(means, quats, scales, viewmat[None], K[None], width, height, 0.3, radii, cn, None,
               vm2, np.zeros_like(d), vcn, None, viewmats_requires_grad=False)
    t["proj_bwd"] = time.perf_counter() - t0

    t0 = time.perf_counter()
    # Adam over all 59 floats per Gaussian (params, m, v), numpy
    for p in (means, quats, log_scales, logit_opac, sh):
        gr = np.zeros_like(p)
        m = np.zeros_like(p)
        v = np.zeros_like(p)
        m = 0.9 * m + 0.1 * gr
        v = 0.999 * v + 0.001 * gr * gr
        _ = p - 1e-3 * m / (np.sqrt(v) + 1e-15)
    t["adam"] = time.perf_counter() - t0
    total = sum(t.values())
    sample = (f"full projection/SH/isect/loss/Adam; rasterize fwd+bwd on 1/{tile_stride} of the "
              f"{n_tiles} tiles scaled by {scale:.1f}; n_isects={len(fids)}")
    return total, t, sample
