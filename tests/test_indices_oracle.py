"""CPU checks of the rasterize_to_indices oracle and the torch `accumulate`
playground (no GPU).

The reference's index kernels are CUDA only, so the oracle is pinned
through the reference's golden rasterizations (tests/golden/raster_garden_*,
produced by the reference Triton kernels): the contributor lists, composited
with `gsplat_hip.accumulate` (plain torch, runs on CPU), must reproduce the
golden images, and every pixel's last contributor must be the Gaussian the
golden `last_ids` names.  The range semantics are checked by splitting the
walk into batches and carrying the transmittance, as the reference's
`_rasterize_to_pixels` does (gsplat/cuda/_torch_impl.py:519-611).
"""

import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import indices_oracle as I
from oracle import surfel_oracle as S

GOLD = os.path.join(ROOT, "tests", "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLD, name if name.endswith(".npz") else name + ".npz")))


def _lists(g, rs=0, re=10**10, trans=None):
    C, N = g["opacities"].shape
    W, H, ts = int(g["width"]), int(g["height"]), int(g["tile_size"])
    if trans is None:
        trans = np.ones((C, H, W), np.float32)
    return I.rasterize_to_indices(0, rs, re, trans, g["means2d"], g["conics"], g["opacities"],
                                  W, H, ts, g["isect_offsets"], g["flatten_ids"])


@pytest.mark.parametrize("name", ["raster_garden_d3_bg", "raster_garden_d4"])
def test_indices_composite_to_golden(name):
    from gsplat_hip import accumulate
    g = _load(name)
    W, H = int(g["width"]), int(g["height"])
    gid, pid, cid = _lists(g)
    assert len(gid) > 1000
    # pixel-major, grouped order
    key = cid * H * W + pid
    assert np.all(np.diff(key) >= 0)
    t = lambda a: torch.from_numpy(np.asarray(a)).double()  # noqa: E731
    rc, ra = accumulate(t(g["means2d"]), t(g["conics"]), t(g["opacities"]), t(g["colors"]),
                        torch.from_numpy(gid), torch.from_numpy(pid), torch.from_numpy(cid), W, H)
    rc, ra = rc.numpy(), ra.numpy()
    if "backgrounds" in g:
        rc = rc + g["backgrounds"][:, None, None, :] * (1 - ra)
    np.testing.assert_allclose(ra, g["render_alphas"], atol=2e-4)
    np.testing.assert_allclose(rc, g["render_colors"], atol=2e-4)


def test_indices_last_contributor_matches_golden_last_ids():
    g = _load("raster_garden_d3_bg")
    C, N = g["opacities"].shape
    W, H = int(g["width"]), int(g["height"])
    gid, pid, cid = _lists(g)
    key = cid * H * W + pid
    last = np.full(C * H * W, -1, np.int64)
    last[key] = gid  # later entries overwrite: the last contributor per pixel
    gold_alpha = g["render_alphas"].reshape(-1)
    gold_last = g["flatten_ids"][g["last_ids"].reshape(-1)].astype(np.int64) % N
    lit = gold_alpha > 0
    agree = (last[lit] == gold_last[lit]).mean()
    # the reference keeps T in log space (L5): a handful of pixels sit on the
    # 1e-4 boundary and may end one record apart
    assert agree > 0.999, agree
    assert np.all(last[~lit] == -1)


def test_indices_ranges_compose():
    """Batches [k, k+1) with the carried transmittance give the same pairs as
    one full walk (the iteration of _rasterize_to_pixels)."""
    g = _load("raster_garden_d4")
    C, N = g["opacities"].shape
    W, H, ts = int(g["width"]), int(g["height"]), int(g["tile_size"])
    full = set(zip(*[a.tolist() for a in _lists(g)]))
    trans = np.ones((C, H, W), np.float32)
    got = set()
    m2, cn, op = g["means2d"], g["conics"], g["opacities"]
    for k in range(0, 64):
        gid, pid, cid = _lists(g, k, k + 1, trans)
        if len(gid) == 0:
            continue
        got |= set(zip(gid.tolist(), pid.tolist(), cid.tolist()))
        # carry T exactly as the kernel does: T *= 1 - alpha per contributor
        px, py = (pid % W).astype(np.float32) + 0.5, (pid // W).astype(np.float32) + 0.5
        dx, dy = m2[cid, gid, 0] - px, m2[cid, gid, 1] - py
        c = cn[cid, gid]
        sig = np.float32(0.5) * (c[:, 0] * dx * dx + c[:, 2] * dy * dy) + c[:, 1] * dx * dy
        al = np.minimum(np.float32(0.999), op[cid, gid] * np.exp(-sig).astype(np.float32))
        for i in range(len(gid)):
            y, x = divmod(int(pid[i]), W)
            trans[cid[i], y, x] = np.float32(trans[cid[i], y, x] * (np.float32(1) - al[i]))
    assert got == full


def test_indices_2dgs_oracle_vs_rasterizer_oracle():
    """2DGS lists composite to the surfel rasterizer oracle's image."""
    from gsplat_hip import accumulate_2dgs
    rng = np.random.default_rng(3)
    C, N, W, H, ts = 1, 300, 48, 40, 16
    g = _load("proj2dgs_random.npz")
    v = g["radii"][0] > 0
    idx = np.nonzero(v)[0][:N]
    N = len(idx)
    m2 = g["means2d"][:1, idx].copy()
    rt = g["ray_transforms"][:1, idx].copy()
    Wg, Hg = int(g["width"]), int(g["height"])
    # crop the projected scene to a small image around its centre
    m2 -= np.array([Wg / 2 - W / 2, Hg / 2 - H / 2], np.float32)
    shift = np.array([[1, 0, -(Wg / 2 - W / 2)], [0, 1, -(Hg / 2 - H / 2)], [0, 0, 1]], np.float32)
    rt = np.einsum("ij,cnjk->cnik", shift, rt).astype(np.float32)
    op = rng.uniform(0.3, 0.95, (C, N)).astype(np.float32)
    col = rng.uniform(0, 1, (C, N, 3)).astype(np.float32)
    nrm = rng.normal(size=(C, N, 3)).astype(np.float32)
    from oracle import gsplat_oracle as O
    radii = g["radii"][:1, idx]
    depths = g["depths"][:1, idx]
    tw, th = (W + ts - 1) // ts, (H + ts - 1) // ts
    _, ids, fids = O.isect_tiles(m2, radii, depths, ts, tw, th)
    offs = O.isect_offset_encode(ids, C, tw, th)
    gid, pid, cid = I.rasterize_to_indices(1, 0, 10**10, np.ones((C, H, W), np.float32), m2, rt,
                                           op, W, H, ts, offs, fids)
    assert len(gid) > 100
    t = lambda a: torch.from_numpy(np.asarray(a)).double()  # noqa: E731
    rc, ra, rn = accumulate_2dgs(t(m2), t(rt.reshape(C, N, 3, 3)), t(op), t(col), t(nrm),
                                 torch.from_numpy(gid), torch.from_numpy(pid),
                                 torch.from_numpy(cid), W, H)
    out = S.raster2dgs_fwd(m2, rt, col, op, nrm, None, None, W, H, ts, offs, fids)
    np.testing.assert_allclose(ra.numpy(), out[1], atol=2e-4)
    np.testing.assert_allclose(rc.numpy(), out[0], atol=2e-4)
    np.testing.assert_allclose(rn.numpy(), out[2], atol=2e-4)
