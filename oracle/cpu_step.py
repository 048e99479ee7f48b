"""CPU baseline for bench.py: one training step of the hot path computed by
the numpy oracle on the host's cores (test infrastructure; only bench.py's
cpu_baseline leg and tests use it).

Parallel over `workers` processes (numpy holds the GIL in this image's
per-tile array loops, so threads do not scale; processes do).  `CpuPool`
starts the workers with the "spawn" method -- bench.py creates it BEFORE its
own process touches the GPU, and the workers import numpy and this package
only -- and hands the arrays over in POSIX shared memory:

  projection, SH, their backward passes and Adam: contiguous chunks of
      Gaussians, one per worker;
  tile intersection (one global sort): the parent, as the reference's torch
      path runs it on one thread;
  rasterize forward: tiles dealt heaviest-first round-robin; each worker
      writes the pixels of its own tiles;
  rasterize backward: same tiles, each worker accumulates its own gradient
      rows [G, 9], summed by the parent (the reference's atomics).

Bounded sample: with `tile_stride` > 1 the rasterizer runs on every
`tile_stride`-th tile and its time is scaled by the number of tiles; with
`tile_stride` == 1 the whole image is rendered.
"""

import math
import multiprocessing as mp
import time
import uuid
from multiprocessing import shared_memory

import numpy as np

from . import gsplat_oracle as O

f32 = np.float32


# ------------------------------------------------------ shared-memory plumbing
class _Shared:
    """Named numpy arrays in POSIX shared memory (owner side)."""

    def __init__(self):
        self.blocks = {}
        self.desc = {}
        self.arrays = {}

    def put(self, name, arr):
        arr = np.ascontiguousarray(arr)
        a = self.empty(name, arr.shape, arr.dtype)
        a[...] = arr
        return a

    def empty(self, name, shape, dtype):
        nbytes = max(int(np.prod(shape)) * np.dtype(dtype).itemsize, 1)
        shm = shared_memory.SharedMemory(create=True, size=nbytes,
                                         name=f"gsplat_cpu_{uuid.uuid4().hex[:12]}")
        self.blocks[name] = shm
        self.desc[name] = (shm.name, tuple(shape), np.dtype(dtype).str)
        a = np.ndarray(shape, dtype, buffer=shm.buf)
        self.arrays[name] = a
        return a

    def close(self):
        self.arrays.clear()
        for shm in self.blocks.values():
            shm.close()
            shm.unlink()
        self.blocks.clear()


_ATTACHED = {}


def _view(desc, names):
    """Worker side: attach (cached) and return the named arrays."""
    out = {}
    for n in names:
        sname, shape, dt = desc[n]
        shm = _ATTACHED.get(sname)
        if shm is None:
            # spawned workers share the parent's resource tracker, where the
            # name is already registered; the parent unlinks it
            shm = _ATTACHED[sname] = shared_memory.SharedMemory(name=sname)
        out[n] = np.ndarray(shape, np.dtype(dt), buffer=shm.buf)
    return out


# ----------------------------------------------------------- worker stages
def _w_forward(job):
    desc, (lo, hi), cfg = job
    a = _view(desc, ["means", "quats", "scales", "viewmat", "K", "sh", "campos", "radii", "m2",
                     "depths", "conics", "colors"])
    radii, m2, d, cn, _ = O.proj_fwd(a["means"][lo:hi], a["quats"][lo:hi], a["scales"][lo:hi],
                                     a["viewmat"][None], a["K"][None], cfg["W"], cfg["H"])
    a["radii"][:, lo:hi] = radii
    a["m2"][:, lo:hi] = m2
    a["depths"][:, lo:hi] = d
    a["conics"][:, lo:hi] = cn
    dirs = (a["means"][lo:hi] - a["campos"])[None].astype(f32)
    col = O.sh_fwd(cfg["deg"], dirs, a["sh"][None, lo:hi], radii > 0)
    a["colors"][:, lo:hi] = np.maximum(col + f32(0.5), 0)
    return True


def _tile_pixels(t, cfg):
    ts, tw, th, W, H = cfg["ts"], cfg["tw"], cfg["th"], cfg["W"], cfg["H"]
    c, rem = divmod(t, tw * th)
    ty, tx = divmod(rem, tw)
    return c, slice(ty * ts, min(H, ty * ts + ts)), slice(tx * ts, min(W, tx * ts + ts))


def _w_raster_fwd(job):
    desc, tiles, cfg = job
    a = _view(desc, ["m2", "conics", "colors", "opac", "offsets", "fids", "rc", "ra", "last"])
    rc, ra, last = O.raster_fwd(a["m2"], a["conics"], a["colors"], a["opac"][None], None,
                                cfg["W"], cfg["H"], cfg["ts"], a["offsets"], a["fids"],
                                tiles=tiles)
    for t in tiles:  # only this worker's pixels
        c, ys, xs = _tile_pixels(t, cfg)
        a["rc"][c, ys, xs] = rc[c, ys, xs]
        a["ra"][c, ys, xs] = ra[c, ys, xs]
        a["last"][c, ys, xs] = last[c, ys, xs]
    return True


def _w_raster_bwd(job):
    desc, tiles, cfg, slot = job
    a = _view(desc, ["m2", "conics", "colors", "opac", "offsets", "fids", "ra", "last", "v_rc",
                     "v_ra", "vrows"])
    vm, vc, vcol, vop, _, _ = O.raster_bwd(a["m2"], a["conics"], a["colors"], a["opac"][None],
                                           None, cfg["W"], cfg["H"], cfg["ts"], a["offsets"],
                                           a["fids"], a["ra"], a["last"], a["v_rc"], a["v_ra"],
                                           tiles=tiles)
    rows = a["vrows"][slot]
    rows[:, 0:2] = vm.reshape(-1, 2)
    rows[:, 2:5] = vc.reshape(-1, 3)
    rows[:, 5:8] = vcol.reshape(-1, 3)
    rows[:, 8] = vop.reshape(-1)
    return True


def _w_backward(job):
    desc, (lo, hi), cfg = job
    a = _view(desc, ["means", "quats", "scales", "viewmat", "K", "sh", "campos", "radii",
                     "conics", "colors", "vsum"])
    v = a["vsum"][lo:hi]
    dirs = (a["means"][lo:hi] - a["campos"])[None].astype(f32)
    vcol = (v[None, :, 5:8] * (a["colors"][:, lo:hi] > 0)).astype(f32)
    masks = a["radii"][:, lo:hi] > 0
    O.sh_bwd(cfg["deg"], dirs, a["sh"][None, lo:hi], vcol, masks, True)
    O.proj_bwd(a["means"][lo:hi], a["quats"][lo:hi], a["scales"][lo:hi], a["viewmat"][None],
               a["K"][None], cfg["W"], cfg["H"], 0.3, a["radii"][:, lo:hi],
               a["conics"][:, lo:hi], None, np.ascontiguousarray(v[None, :, 0:2]),
               np.zeros((1, hi - lo), f32), np.ascontiguousarray(v[None, :, 2:5]), None,
               viewmats_requires_grad=False)
    return True


def _w_adam(job):
    """torch.optim.Adam's update over this chunk's 59 floats per Gaussian
    (parameters, both moments; gradients as computed, zero-filled here)."""
    desc, (lo, hi), cfg = job
    a = _view(desc, ["means", "quats", "scales", "opac", "sh"])
    for k in ("means", "quats", "scales", "opac", "sh"):
        p = a[k][lo:hi]
        gr = np.zeros_like(p)
        m = np.zeros_like(p)
        v = np.zeros_like(p)
        m = 0.9 * m + 0.1 * gr
        v = 0.999 * v + 0.001 * gr * gr
        _ = p - 1e-3 * m / (np.sqrt(v) + 1e-15)
    return True


def _w_noop(_):
    return True


def _chunks(n, k):
    b = np.linspace(0, n, k + 1).astype(np.int64)
    return [(int(b[i]), int(b[i + 1])) for i in range(k) if b[i + 1] > b[i]]


# ------------------------------------------------------------------- driver
class CpuPool:
    """`workers` spawned numpy processes.  Create it before the calling
    process initialises the GPU; call `close()` when done."""

    def __init__(self, workers):
        self.workers = max(1, int(workers))
        self.pool = None
        if self.workers > 1:
            self.pool = mp.get_context("spawn").Pool(self.workers)
            self.pool.map(_w_noop, range(self.workers))  # interpreters up now

    def map(self, fn, jobs):
        if self.pool is None:
            return [fn(j) for j in jobs]
        return self.pool.map(fn, jobs, chunksize=1)

    def close(self):
        if self.pool is not None:  # workers exit: their mappings go with them
            self.pool.close()
            self.pool.join()
            self.pool = None
        for shm in _ATTACHED.values():
            shm.close()
        _ATTACHED.clear()


def cpu_train_step(means, quats, log_scales, logit_opac, sh, viewmat, K, width, height,
                   target, tile_stride=1, sh_degree=3, tile_size=16, pool=None):
    """Returns (seconds for the full step (scaled when sampled), breakdown
    dict, sample description).  `pool`: a CpuPool (None: one process)."""
    own = pool is None
    if own:
        pool = CpuPool(1)
    nw = pool.workers
    S = _Shared()
    try:
        t = {}
        C = 1
        N = means.shape[0]
        tw, th = math.ceil(width / tile_size), math.ceil(height / tile_size)
        cfg = {"W": width, "H": height, "deg": sh_degree, "ts": tile_size, "tw": tw, "th": th}
        parts = _chunks(N, nw)
        # inputs (the parameters as the trainer holds them, activated below)
        for k, v in (("means", means), ("quats", quats), ("sh", sh), ("viewmat", viewmat),
                     ("K", K)):
            S.put(k, np.asarray(v, f32))
        S.put("campos", np.linalg.inv(np.asarray(viewmat, np.float64))[:3, 3].astype(f32))
        for k, shp, dt in (("radii", (C, N), np.int32), ("m2", (C, N, 2), f32),
                           ("depths", (C, N), f32), ("conics", (C, N, 3), f32),
                           ("colors", (C, N, 3), f32)):
            S.empty(k, shp, dt)

        t0 = time.perf_counter()
        S.put("scales", np.exp(log_scales).astype(f32))
        S.put("opac", (1.0 / (1.0 + np.exp(-logit_opac))).astype(f32))
        pool.map(_w_forward, [(S.desc, r, cfg) for r in parts])
        t["proj_sh_fwd"] = time.perf_counter() - t0

        A = S.arrays
        t0 = time.perf_counter()
        _, ids, fids = O.isect_tiles(A["m2"], A["radii"], A["depths"], tile_size, tw, th)
        off = O.isect_offset_encode(ids, C, tw, th)
        S.put("offsets", off)
        S.put("fids", fids.astype(np.int64))
        t["isect"] = time.perf_counter() - t0

        n_tiles = C * tw * th
        tiles = list(range(0, n_tiles, max(1, tile_stride)))
        scale = n_tiles / len(tiles)
        # heaviest tiles dealt first, round-robin, so the workers finish together
        cnt = np.diff(np.append(off.reshape(-1).astype(np.int64), len(fids)))[tiles]
        order = [tiles[i] for i in np.argsort(-cnt, kind="stable")]
        per = max(1, min(nw * 8, len(order)))
        tsets = [order[i::per] for i in range(per)]
        rc = S.empty("rc", (C, height, width, 3), f32)
        ra = S.empty("ra", (C, height, width, 1), f32)
        S.empty("last", (C, height, width), np.int32)
        rc[...] = 0
        ra[...] = 0
        t0 = time.perf_counter()
        pool.map(_w_raster_fwd, [(S.desc, ts, cfg) for ts in tsets])
        t["raster_fwd"] = (time.perf_counter() - t0) * scale

        t0 = time.perf_counter()
        # L1 part of the loss gradient (the SSIM part costs the same order; glue)
        S.put("v_rc", (np.sign(rc - np.asarray(target, f32)[None]) * (0.8 / rc.size)).astype(f32))
        S.put("v_ra", np.zeros_like(ra))
        t["loss"] = time.perf_counter() - t0

        bsets = [order[i::nw] for i in range(nw)]
        vrows = S.empty("vrows", (len(bsets), C * N, 9), f32)
        t0 = time.perf_counter()
        pool.map(_w_raster_bwd, [(S.desc, ts, cfg, i) for i, ts in enumerate(bsets)])
        S.put("vsum", vrows.sum(0))
        t["raster_bwd"] = (time.perf_counter() - t0) * scale

        t0 = time.perf_counter()
        pool.map(_w_backward, [(S.desc, r, cfg) for r in parts])
        t["sh_proj_bwd"] = time.perf_counter() - t0

        t0 = time.perf_counter()
        pool.map(_w_adam, [(S.desc, r, cfg) for r in parts])
        t["adam"] = time.perf_counter() - t0
        total = sum(t.values())
        if len(tiles) == n_tiles:
            what = f"rasterize fwd+bwd on all {n_tiles} tiles"
        else:
            what = (f"rasterize fwd+bwd on 1/{tile_stride} of the {n_tiles} tiles scaled by "
                    f"{scale:.1f}")
        sample = (f"one full train step on {nw} worker processes: projection/SH/isect/"
                  f"loss(L1)/Adam on all {N} Gaussians; {what}; n_isects={len(fids)}")
        return total, t, sample
    finally:
        S.close()
        if own:
            pool.close()
