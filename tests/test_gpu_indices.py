"""GPU parity of rasterize_to_indices_in_range{,_2dgs} (csrc/indices.hip,
through the C ABI) against the indices oracle, and of the iterative torch
rasterizer built on it (`_rasterize_to_pixels`) against the fused HIP
rasterizer -- the reference's own check (tests/test_basic.py:440-533, same
tolerances).  Lists are integer outputs: they must be identical up to the
threshold flips described in test_gpu_parity.close_most (a pixel whose alpha
or T sits within fp32 rounding of 1/255 or 1e-4)."""

import math

import numpy as np
import pytest
import torch

from oracle import indices_oracle as I
from test_gpu_parity import DEV, T, close_most
from test_indices_oracle import _load
from test_surfel_oracle import surfel_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def _per_pixel(gid, pid, cid, H, W):
    key = (cid.astype(np.int64) * H * W + pid)
    out = {}
    for k, g in zip(key.tolist(), gid.tolist()):
        out.setdefault(k, []).append(g)
    return out


def same_lists(got, want, H, W, max_frac=1e-3):
    got = [x.cpu().numpy() if isinstance(x, torch.Tensor) else x for x in got]
    for a in got:
        assert a.dtype == np.int64
    key = got[2] * H * W + got[1]
    assert np.all(np.diff(key) >= 0), "not pixel-major"
    if all(np.array_equal(a, b) for a, b in zip(got, want)):
        return
    pa, pb = _per_pixel(*got, H, W), _per_pixel(*want, H, W)
    bad = sum(pa.get(k) != pb.get(k) for k in set(pa) | set(pb))
    assert bad <= max(2, max_frac * len(pb)), f"{bad} of {len(pb)} pixels differ"


def _retile(g, ts):
    """The fixture's Gaussians re-binned to tile_size `ts` (radius 3 sigma of
    the conic's covariance, fixed pseudo-random depths) so that tiles span
    several batches of ts*ts records."""
    from oracle import gsplat_oracle as O
    C, N = g["opacities"].shape
    W, H = int(g["width"]), int(g["height"])
    a, b, c = (g["conics"][..., k].astype(np.float64) for k in range(3))
    det = a * c - b * b
    ok = det > 0
    det = np.where(ok, det, 1.0)
    tr = (a + c) / det  # trace of the covariance
    lam = 0.5 * tr + np.sqrt(np.maximum(0.25 * tr * tr - 1 / det, 0))
    radii = np.where(ok, np.ceil(3 * np.sqrt(lam)), 0).astype(np.int32)
    depths = np.random.default_rng(1).uniform(1, 5, (C, N)).astype(np.float32)
    tw, th = math.ceil(W / ts), math.ceil(H / ts)
    _, ids, fids = O.isect_tiles(g["means2d"], radii, depths, ts, tw, th)
    return O.isect_offset_encode(ids, C, tw, th), fids


@pytest.mark.parametrize("name", ["raster_garden_d3_bg", "raster_garden_d8_bg"])
@pytest.mark.parametrize("ts,rng_", [(16, (0, 10**10)), (4, (0, 10**10)), (4, (0, 1)),
                                     (4, (1, 3))])
def test_indices_3dgs_vs_oracle(name, ts, rng_):
    from gsplat_hip import rasterize_to_indices_in_range
    g = _load(name)
    C, N = g["opacities"].shape
    W, H = int(g["width"]), int(g["height"])
    off, fids = (g["isect_offsets"], g["flatten_ids"]) if ts == 16 else _retile(g, ts)
    trans = np.random.default_rng(0).uniform(0.2, 1.0, (C, H, W)).astype(np.float32)
    if rng_[0] == 0:
        trans[:] = 1.0
    got = rasterize_to_indices_in_range(rng_[0], rng_[1], T(trans), T(g["means2d"]),
                                        T(g["conics"]), T(g["opacities"]), W, H, ts, T(off),
                                        T(fids))
    want = I.rasterize_to_indices(0, rng_[0], rng_[1], trans, g["means2d"], g["conics"],
                                  g["opacities"], W, H, ts, off, fids)
    assert len(want[0]) > 100
    same_lists(got, want, H, W)


@pytest.mark.parametrize("seed,C", [(0, 1), (1, 2)])
def test_indices_2dgs_vs_oracle(seed, C):
    from gsplat_hip import rasterize_to_indices_in_range_2dgs
    sc = surfel_scene(seed, N=300, W=70, H=52, D=3, bg=False, C=C)
    N = sc["m2"].shape[1]
    trans = np.ones((C, sc["H"], sc["W"]), np.float32)
    got = rasterize_to_indices_in_range_2dgs(0, 10**10, T(trans), T(sc["m2"]),
                                             T(sc["rt"]).view(C, N, 3, 3), T(sc["opac"]),
                                             sc["W"], sc["H"], sc["ts"], T(sc["off"]),
                                             T(sc["fids"]))
    want = I.rasterize_to_indices(1, 0, 10**10, trans, sc["m2"], sc["rt"], sc["opac"], sc["W"],
                                  sc["H"], sc["ts"], sc["off"], sc["fids"])
    assert len(want[0]) > 100
    same_lists(got, want, sc["H"], sc["W"])


def test_indices_empty_and_out_of_range():
    from gsplat_hip import rasterize_to_indices_in_range
    g = _load("raster_garden_d4")
    C, N = g["opacities"].shape
    W, H, ts = int(g["width"]), int(g["height"]), int(g["tile_size"])
    args = (T(np.ones((C, H, W), np.float32)), T(g["means2d"]), T(g["conics"]),
            T(g["opacities"]), W, H, ts)
    gid, pid, cid = rasterize_to_indices_in_range(10**6, 10**6 + 5, *args,
                                                  T(g["isect_offsets"]), T(g["flatten_ids"]))
    assert gid.numel() == 0 and pid.numel() == 0 and cid.numel() == 0
    empty_off = torch.zeros_like(T(g["isect_offsets"]))
    gid, _, _ = rasterize_to_indices_in_range(0, 10**10, *args, empty_off,
                                              torch.empty(0, dtype=torch.int32, device=DEV))
    assert gid.numel() == 0


def _pipeline(channels, seed=42, C=2, W=120, H=90, N=2000):
    from gsplat_hip import fully_fused_projection, isect_offset_encode, isect_tiles
    g = torch.Generator().manual_seed(seed)
    means = (torch.randn(N, 3, generator=g) * torch.tensor([1.0, 0.8, 0.5])
             + torch.tensor([0, 0, 4.0])).to(DEV)
    quats = torch.randn(N, 4, generator=g).to(DEV)
    scales = (torch.rand(N, 3, generator=g) * 0.06 + 0.01).to(DEV)
    opac = torch.rand(N, generator=g).to(DEV)
    vms = torch.eye(4).repeat(C, 1, 1)
    vms[:, 0, 3] = torch.arange(C) * 0.2
    K = torch.tensor([[110.0, 0, W / 2], [0, 110.0, H / 2], [0, 0, 1]]).repeat(C, 1, 1)
    radii, m2, depths, conics, _ = fully_fused_projection(means, None, quats, scales,
                                                          vms.to(DEV), K.to(DEV), W, H)
    ts = 16 if channels <= 32 else 4
    tw, th = math.ceil(W / ts), math.ceil(H / ts)
    _, ids, fids = isect_tiles(m2, radii, depths, ts, tw, th)
    off = isect_offset_encode(ids, C, tw, th)
    colors = torch.randn(C, N, channels, generator=g).to(DEV)
    bgs = torch.rand(C, channels, generator=g).to(DEV)
    return m2, conics, colors, opac.repeat(C, 1), bgs, W, H, ts, off, fids


@pytest.mark.parametrize("channels", [3, 32, 128])
def test_torch_rasterize_to_pixels_matches_fused(channels):
    """tests/test_basic.py:440-533 on this backend: the iterative rasterizer
    (index lists + accumulate, autograd) against the fused HIP kernels."""
    from gsplat_hip import rasterize_to_pixels
    from gsplat_hip._wrapper_indices import _rasterize_to_pixels
    m2, cn, col, op, bg, W, H, ts, off, fids = _pipeline(channels)
    leaves = [x.detach().clone().requires_grad_(True) for x in (m2, cn, col, op, bg)]
    rc, ra = rasterize_to_pixels(*leaves[:4], W, H, ts, off, fids, backgrounds=leaves[4])
    _rc, _ra = _rasterize_to_pixels(*leaves[:4], W, H, ts, off, fids, backgrounds=leaves[4],
                                    batch_per_iter=3)
    # the reference's tolerances (torch defaults for the images), up to
    # threshold flips (exp2 vs exp for alpha in the two paths)
    close_most(rc, _rc, 1.3e-6, 1e-5, "colors", max_frac=1e-4)
    close_most(ra, _ra, 1.3e-6, 1e-5, "alphas", max_frac=1e-4)
    vrc, vra = torch.randn_like(rc), torch.randn_like(ra)
    ga = torch.autograd.grad((rc * vrc).sum() + (ra * vra).sum(), leaves)
    gb = torch.autograd.grad((_rc * vrc).sum() + (_ra * vra).sum(), leaves)
    for a, b, tol, what in zip(ga, gb, (5e-3, 1e-3, 1e-3, 2e-3, 1e-3),
                               ("means2d", "conics", "colors", "opacities", "backgrounds")):
        close_most(a, b, tol, tol, what, max_frac=1e-3, rows=a.dim() > 2)


def test_torch_rasterize_to_pixels_2dgs_matches_fused():
    """tests/test_2dgs.py:234-330 on this backend (forward images)."""
    from gsplat_hip import rasterize_to_pixels_2dgs
    from gsplat_hip._wrapper_indices import _rasterize_to_pixels_2dgs
    sc = surfel_scene(5, N=300, W=70, H=52, D=3, bg=True, C=1)
    N = sc["m2"].shape[1]
    m2, rt = T(sc["m2"]), T(sc["rt"]).view(1, N, 3, 3)
    col, op, nr, bg = T(sc["colors"]), T(sc["opac"]), T(sc["nr"]), T(sc["bg"])
    off, fids = T(sc["off"]), T(sc["fids"])
    rc, ra, rn, _, _ = rasterize_to_pixels_2dgs(m2, rt, col, op, nr, torch.zeros_like(m2),
                                                sc["W"], sc["H"], sc["ts"], off, fids,
                                                backgrounds=bg)
    _rc, _ra, _rn = _rasterize_to_pixels_2dgs(m2, rt, col, nr, op, sc["W"], sc["H"], sc["ts"],
                                              off, fids, backgrounds=bg, batch_per_iter=2)
    close_most(ra, _ra, 1e-4, 1e-4, "alphas", max_frac=5e-3)
    close_most(rc, _rc, 1e-4, 1e-4, "colors", max_frac=5e-3)
    close_most(rn, _rn, 1e-4, 1e-4, "normals", max_frac=5e-3)
