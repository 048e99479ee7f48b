"""CPU oracle for rasterize_to_indices_in_range{,_2dgs} -- TEST INFRASTRUCTURE
ONLY (imported by tests/ only; the product never touches it).

numpy float32 restatement of the reference CUDA kernels
  rasterize_to_indices_3dgs_kernel  gsplat/cuda/csrc/RasterizeToIndices3DGS.cu:14-185
  rasterize_to_indices_2dgs_kernel  gsplat/cuda/csrc/RasterizeToIndices2DGS.cu:14-200
and their two-pass driver (gsplat/cuda/csrc/Rasterization.cpp:224-296):
per pixel, walk the tile's records in batches [range_start, range_end) of
ts*ts, skip sigma < 0 / alpha < 1/255 (2DGS also a zero ray cross product),
stop before the record that would bring T <= 1e-4, and emit
(flatten_id % N, c*H*W + pixel) in pixel-major, front-to-back order.

Parity: unpinned against the reference's own output (the kernels are CUDA
only and the reference's torch consumer needs nerfacc, absent here); the
oracle shares the alpha algebra with the pinned rasterizer oracles
(gsplat_oracle.raster_fwd, surfel_oracle._eval), and tests check that the
lists composite to the pinned rasterizers' images.
"""

import numpy as np

from .surfel_oracle import _eval

f32 = np.float32
ALPHA_MIN, ALPHA_MAX, T_MIN = f32(1.0 / 255.0), f32(0.999), f32(1e-4)


def _alpha3(rec, px, py):
    x, y, a, b, c, op = rec
    dx, dy = x - px, y - py
    with np.errstate(all="ignore"):
        sig = f32(0.5) * (a * dx * dx + c * dy * dy) + b * dx * dy
        al = np.minimum(ALPHA_MAX, op * np.exp(-sig).astype(f32))
    return al, ~(sig < 0) & ~(al < ALPHA_MIN)


def rasterize_to_indices(kind, range_start, range_end, transmittances, means2d, shape,
                         opacities, W, H, ts, offsets, flatten_ids):
    """Returns (gaussian_ids, pixel_ids, camera_ids), int64 [M] each."""
    offsets = np.asarray(offsets)
    C, th, tw = offsets.shape
    N = np.asarray(means2d).shape[1]
    m2 = np.asarray(means2d, f32).reshape(-1, 2)
    sh = np.asarray(shape, f32).reshape(C * N, -1)
    op = np.asarray(opacities, f32).reshape(-1)
    fids = np.asarray(flatten_ids, np.int64)
    trans = np.asarray(transmittances, f32)
    flat = offsets.reshape(-1).astype(np.int64)
    ends = np.append(flat[1:], len(fids))
    bs = ts * ts
    ly, lx = np.meshgrid(np.arange(ts), np.arange(ts), indexing="ij")
    lists = {}  # global pixel index -> list of gaussian ids
    for t in range(C * th * tw):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        pyi, pxi = (ly + ty * ts).reshape(-1), (lx + tx * ts).reshape(-1)
        inside = (pyi < H) & (pxi < W)
        pyi, pxi = pyi[inside], pxi[inside]
        if len(pyi) == 0:
            continue
        px, py = pxi.astype(f32) + f32(0.5), pyi.astype(f32) + f32(0.5)
        s, e = flat[t], ends[t]
        nb = (e - s + bs - 1) // bs
        r0 = s + bs * min(range_start, nb)
        r1 = min(e, s + bs * min(range_end, nb))
        T = trans[c, pyi, pxi].copy()
        done = np.zeros(len(pyi), bool)
        pix = (c * H + pyi) * W + pxi
        out = [[] for _ in range(len(pyi))]
        for i in range(r0, r1):
            if done.all():
                break
            g = fids[i]
            if kind == 0:
                al, ok = _alpha3((m2[g, 0], m2[g, 1], sh[g, 0], sh[g, 1], sh[g, 2], op[g]), px, py)
            else:
                ev = _eval(sh[g], m2[g, 0], m2[g, 1], op[g], px, py)
                al, ok = ev["alpha"], ev["ok"]
            ok &= ~done
            nT = (T * (f32(1.0) - al)).astype(f32)
            stop = ok & (nT <= T_MIN)
            done |= stop
            emit = ok & ~stop
            for k in np.nonzero(emit)[0]:
                out[k].append(g % N)
            T = np.where(emit, nT, T)
        for k in range(len(pyi)):
            if out[k]:
                lists[int(pix[k])] = out[k]
    keys = sorted(lists)
    gid = np.array([g for k in keys for g in lists[k]], np.int64)
    idx = np.array([k for k in keys for _ in lists[k]], np.int64)
    return gid, idx % (W * H), idx // (W * H)
