"""GPU parity: the HIP path (through the C ABI) against the reference goldens
and the CPU oracle.  Tolerances follow the reference's own tests
(triton_tests/test_fused_proj.py:116-162, test_sh.py:25-37,
test_isect.py:86-89 [exact], test_ras2pix.py:132-161)."""

import math

import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def T(x, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    return t if dtype is None else t.to(dtype)


def close(a, b, rtol, atol, what=""):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


def close_most(a, b, rtol, atol, what="", max_frac=1e-4, min_count=2, rows=False,
               out_bound=None):
    """allclose up to a handful of threshold flips: a Gaussian whose alpha is
    within float rounding of 1/255 (or a pixel whose T is within rounding of
    1e-4) can land on the other side of the cut in two correct fp32
    implementations (different FMA contraction / exp).  At most
    max(min_count, max_frac * n) elements -- or, with rows=True, rows of the
    last axis (all gradient components of one Gaussian) -- may exceed the
    tolerance, and each of those by at most `out_bound` in absolute value.

    Default bound: a flip adds or drops one Gaussian of alpha ~1/255 at one
    pixel, which moves that pixel's colour / alpha by <= 1/255 * |c| and every
    later contribution by a factor (1 - 1/255): <= 2/255 of the largest value,
    taken as 0.01 * max|b| (+ atol).  Gradient call sites pass their own."""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad_el = ~np.isclose(a, b, rtol=rtol, atol=atol)
    bad = bad_el
    if rows and bad.ndim > 1:
        bad = bad.reshape(-1, bad.shape[-1]).any(-1)
    allowed = max(min_count, int(max_frac * bad.size))
    diff = np.abs(a.astype(np.float64) - b)
    assert bad.sum() <= allowed, (
        f"{what}: {bad.sum()} of {bad.size} {'rows' if rows else 'elements'} outside "
        f"rtol={rtol} atol={atol} (allowed {allowed}); max abs diff {diff.max()}")
    if out_bound is None:
        out_bound = 0.01 * float(np.abs(b).max(initial=0.0)) + atol
    if bad_el.any():
        worst = float(diff[bad_el].max())
        assert worst <= out_bound, (
            f"{what}: an outlier is off by {worst}, beyond the one-flip bound {out_bound}")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401  (fails loudly if the .so is missing)


# -------------------------------------------------------------- projection
PROJ = ["proj_garden", "proj_garden_comp", "proj_synth", "proj_synth_comp"]


@pytest.mark.parametrize("name", PROJ)
def test_projection_vs_reference(name):
    import gsplat_hip
    g = load_golden(name)
    comp = "comps" in g
    m, q, s, vm = (T(g[k]).requires_grad_(True) for k in ("means", "quats", "scales", "viewmats"))
    radii, m2, d, cn, cp = gsplat_hip.fully_fused_projection(
        m, None, q, s, vm, T(g["Ks"]), int(g["width"]), int(g["height"]), eps2d=float(g["eps2d"]),
        near_plane=float(g["near"]), far_plane=float(g["far"]),
        radius_clip=float(g["radius_clip"]), calc_compensations=comp)
    assert torch.equal(radii.cpu(), torch.from_numpy(g["radii"]))
    v = radii.cpu().numpy() > 0
    close(m2.detach().cpu().numpy()[v], g["means2d"][v], 1e-4, 1e-4, "means2d")
    close(d, g["depths"], 1e-5, 1e-5, "depths")
    close(cn.detach().cpu().numpy()[v], g["conics"][v], 1e-4, 1e-5, "conics")
    if comp:
        close(cp.detach().cpu().numpy()[v], g["comps"][v], 5e-4, 1e-3, "comps")
    loss = (m2 * T(g["v_means2d"])).sum() + (d * T(g["v_depths"])).sum() \
        + (cn * T(g["v_conics"])).sum()
    if comp:
        loss = loss + (cp * T(g["v_comps"])).sum()
    gm, gq, gs, gv = torch.autograd.grad(loss, (m, q, s, vm))
    close(gm, g["v_means"], 1e-3, 1e-3, "v_means")
    close(gq, g["v_quats"], 5e-3, 5e-3, "v_quats")
    close(gs, g["v_scales"], 5e-2, 5e-2, "v_scales")
    ref = g["v_viewmats"]
    fin = np.isfinite(ref)  # the reference's v_viewmats can be NaN-poisoned (L22)
    close(gv.cpu().numpy()[fin], ref[fin], 1e-4, 5e-3, "v_viewmats")


# -------------------------------------------------------------------- SH
@pytest.mark.parametrize("deg", range(5))
def test_sh_vs_reference(deg):
    import gsplat_hip
    g = load_golden(f"sh_deg{deg}")
    cf = T(g["coeffs"]).requires_grad_(True)
    dr = T(g["dirs"]).requires_grad_(True)
    col = gsplat_hip.spherical_harmonics(deg, dr, cf, masks=T(g["masks"]))
    close(col, g["colors"], 1e-4, 1e-4, "colors")
    gc, gd = torch.autograd.grad((col * T(g["v_colors"])).sum(), (cf, dr))
    close(gc, g["v_coeffs"], 1e-4, 1e-4, "v_coeffs")
    if deg > 0:
        close(gd, g["v_dirs"], 1e-4, 1e-4, "v_dirs")


def test_sh_broadcast_coeffs_match_materialised():
    import gsplat_hip
    torch.manual_seed(0)
    C, N = 3, 777
    sh = torch.randn(N, 16, 3, device=DEV, requires_grad=True)
    dirs = torch.randn(C, N, 3, device=DEV)
    masks = torch.rand(C, N, device=DEV) > 0.3
    a = gsplat_hip.spherical_harmonics(3, dirs, sh.expand(C, -1, -1, -1), masks=masks)
    b = gsplat_hip.spherical_harmonics(3, dirs, sh.expand(C, -1, -1, -1).contiguous(), masks=masks)
    assert torch.equal(a, b)
    ga, = torch.autograd.grad(a.sum(), sh)
    gb, = torch.autograd.grad(b.sum(), sh)
    close(ga, gb, 1e-6, 1e-6)


# ----------------------------------------------------------------- isect
@pytest.fixture(params=["tile_first", "depth_first", "full"])
def isect_mode(request, monkeypatch):
    """Run an isect test under both sort strategies of _wrapper.isect_tiles."""
    from gsplat_hip import _wrapper
    monkeypatch.setattr(_wrapper, "ISECT_SORT", request.param)
    return request.param


def _isect(m2, r, d, ts, tw, th):
    """isect_tiles plus the tile offsets the sorted emission writes with the
    isects (None for the strategies that do not)."""
    from gsplat_hip import _wrapper
    p = _wrapper.isect_tiles_begin(m2, r, d, ts, tw, th)
    tpg, ids, fids = p.finish(sort=True)
    return tpg, ids, fids, p.offsets


def _check_offsets(off, ids, C, tw, th):
    """Offsets written with the isects == isect_offset_encode of the ids."""
    import gsplat_hip
    if off is not None:
        assert torch.equal(off, gsplat_hip.isect_offset_encode(ids, C, tw, th))


@pytest.mark.parametrize("name", ["isect_garden_t16", "isect_garden_t4", "isect_pow2_c2"])
def test_isect_bit_exact_vs_reference(name, isect_mode):
    import gsplat_hip
    g = load_golden(name)
    ts, tw, th, C = (int(g[k]) for k in ("tile_size", "tile_width", "tile_height", "C"))
    tpg, ids, fids, off_w = _isect(T(g["means2d"]), T(g["radii"]), T(g["depths"]), ts, tw, th)
    assert np.array_equal(tpg.cpu().numpy(), g["tiles_per_gauss"])
    assert np.array_equal(ids.cpu().numpy(), g["isect_ids"])
    assert np.array_equal(fids.cpu().numpy(), g["flatten_ids"])
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    assert np.array_equal(off.cpu().numpy(), g["isect_offsets"])
    if off_w is not None:
        assert np.array_equal(off_w.cpu().numpy(), g["isect_offsets"])


def test_isect_edge_cases(isect_mode):
    import gsplat_hip
    from oracle import gsplat_oracle as O
    # empty input, all-invalid input, single isect
    for C, N in ((1, 0), (2, 5)):
        m2 = torch.zeros(C, N, 2, device=DEV)
        r = torch.zeros(C, N, dtype=torch.int32, device=DEV)
        d = torch.ones(C, N, device=DEV)
        tpg, ids, fids, off_w = _isect(m2, r, d, 16, 4, 3)
        assert ids.numel() == 0 and fids.numel() == 0 and not tpg.any()
        assert off_w is None or (off_w.shape == (C, 3, 4) and not off_w.any())
        off = gsplat_hip.isect_offset_encode(ids, C, 4, 3)
        assert off.shape == (C, 3, 4) and not off.any()
    ids = torch.tensor([(2 << 32) | 7], dtype=torch.int64, device=DEV)
    off = gsplat_hip.isect_offset_encode(ids, 1, 3, 2)
    assert off.flatten().tolist() == O.isect_offset_encode(ids.cpu().numpy(), 1, 3, 2).reshape(-1).tolist()


def test_isect_random_vs_oracle_large_radii(isect_mode):
    """Ragged input: huge and tiny radii, off-screen means, C=3, exact."""
    import gsplat_hip
    from oracle import gsplat_oracle as O
    rng = np.random.default_rng(1)
    C, N, W, H, ts = 3, 3000, 333, 211, 16
    tw, th = math.ceil(W / ts), math.ceil(H / ts)
    m2 = rng.uniform(-60, 400, (C, N, 2)).astype(np.float32)
    r = rng.choice([0, 1, 2, 5, 17, 90, 300], (C, N)).astype(np.int32)
    d = rng.uniform(0.05, 50, (C, N)).astype(np.float32)
    d[0, :50] = d[0, 50:100]  # depth ties -> stability matters
    tpg, ids, fids, off_w = _isect(T(m2), T(r), T(d), ts, tw, th)
    otpg, oids, ofids = O.isect_tiles(m2, r, d, ts, tw, th)
    assert np.array_equal(tpg.cpu().numpy(), otpg)
    assert np.array_equal(ids.cpu().numpy(), oids)
    assert np.array_equal(fids.cpu().numpy(), ofids)
    _check_offsets(off_w, ids, C, tw, th)
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    assert np.array_equal(off.cpu().numpy(), O.isect_offset_encode(oids, C, tw, th))


def test_isect_huge_gaussians_vs_oracle(isect_mode):
    """Gaussians covering thousands of tiles (the grid-wide emission path,
    > 1024 tiles), many of them adjacent in depth order, some with negative
    depth (all-ones key), mixed with small ones: exact."""
    import gsplat_hip
    from oracle import gsplat_oracle as O
    rng = np.random.default_rng(7)
    C, N, W, H, ts = 2, 2500, 1100, 900, 16
    tw, th = math.ceil(W / ts), math.ceil(H / ts)
    m2 = rng.uniform(-100, 1200, (C, N, 2)).astype(np.float32)
    r = rng.choice([0, 2, 9, 40, 200], (C, N)).astype(np.int32)
    d = rng.uniform(1.0, 50, (C, N)).astype(np.float32)
    huge = rng.choice(N, 150, replace=False)
    r[:, huge] = rng.integers(300, 5000, (C, 150))
    d[:, huge] = rng.uniform(0.01, 0.02, (C, 150))  # nearest: adjacent after the depth sort
    d[0, huge[:10]] = -1.0
    tpg, ids, fids, off_w = _isect(T(m2), T(r), T(d), ts, tw, th)
    otpg, oids, ofids = O.isect_tiles(m2, r, d, ts, tw, th)
    _check_offsets(off_w, ids, C, tw, th)
    assert int((otpg > 1024).sum()) >= 100
    assert np.array_equal(tpg.cpu().numpy(), otpg)
    assert np.array_equal(ids.cpu().numpy(), oids)
    assert np.array_equal(fids.cpu().numpy(), ofids)


@pytest.mark.parametrize("C,tw,th", [(1, 4, 4), (2, 5, 3), (4, 8, 8)])
def test_isect_negative_and_tied_depths(isect_mode, C, tw, th):
    """Negative depths (sign-extended ids that land in the all-ones (cam, tile)
    key), +-0.0, many exact ties, and grids whose last tile id is all ones."""
    import gsplat_hip
    from oracle import gsplat_oracle as O
    rng = np.random.default_rng(C * 100 + tw)
    ts, N = 16, 700
    m2 = rng.uniform(-20, 16 * max(tw, th) + 20, (C, N, 2)).astype(np.float32)
    r = rng.choice([0, 3, 9, 30, 70], (C, N)).astype(np.int32)
    d = rng.choice(np.array([-2.5, -1e-3, -0.0, 0.0, 0.5, 0.5, 1.0, 3.0, 1e6], np.float32), (C, N))
    d = np.where(rng.random((C, N)) < 0.3, rng.uniform(-5, 5, (C, N)), d).astype(np.float32)
    tpg, ids, fids, off_w = _isect(T(m2), T(r), T(d), ts, tw, th)
    otpg, oids, ofids = O.isect_tiles(m2, r, d, ts, tw, th)
    _check_offsets(off_w, ids, C, tw, th)
    assert np.array_equal(tpg.cpu().numpy(), otpg)
    assert np.array_equal(ids.cpu().numpy(), oids)
    assert np.array_equal(fids.cpu().numpy(), ofids)


@pytest.mark.parametrize("N,rmax", [(200_000, 60), (1_000_000, 12)])
def test_isect_sort_strategies_agree_large(N, rmax):
    """Both strategies on an M2-sized random workload (~1M isects); the
    second size has > 2^20 visible Gaussians (the 16-items-per-thread tiles
    of the 11-bit depth sort)."""
    import gsplat_hip
    from gsplat_hip import _wrapper
    g = torch.Generator(device=DEV).manual_seed(3)
    C, ts, tw, th = 2, 16, 120, 68
    m2 = torch.rand(C, N, 2, device=DEV, generator=g) * torch.tensor([tw * ts, th * ts], device=DEV)
    r = (torch.rand(C, N, device=DEV, generator=g) ** 4 * rmax).int()
    d = torch.rand(C, N, device=DEV, generator=g) * 10
    d[:, ::7] = 1.0  # ties
    old = _wrapper.ISECT_SORT
    try:
        out = {}
        for mode in ("tile_first", "depth_first", "full"):
            _wrapper.ISECT_SORT = mode
            out[mode] = gsplat_hip.isect_tiles(m2, r, d, ts, tw, th)
    finally:
        _wrapper.ISECT_SORT = old
    for mode in ("tile_first", "depth_first"):
        for a, b in zip(out[mode], out["full"]):
            assert torch.equal(a, b), mode
    assert out["full"][1].numel() > 100_000


# ------------------------------------------------------------ rasterize
RASTER = ["raster_garden_d3_bg", "raster_garden_d4", "raster_garden_d8_bg"]


@pytest.mark.parametrize("name", RASTER)
def test_raster_vs_reference(name):
    import gsplat_hip
    g = load_golden(name)
    use_bg = "backgrounds" in g
    m2, cn, cl, op = (T(g[k]).requires_grad_(True) for k in ("means2d", "conics", "colors",
                                                             "opacities"))
    bg = T(g["backgrounds"]).requires_grad_(True) if use_bg else None
    rc, ra = gsplat_hip.rasterize_to_pixels(m2, cn, cl, op, int(g["width"]), int(g["height"]),
                                            int(g["tile_size"]), T(g["isect_offsets"]),
                                            T(g["flatten_ids"]), backgrounds=bg, absgrad=True)
    close(ra, g["render_alphas"], 1.3e-6 * 10, 1e-5, "alphas")
    close(rc, g["render_colors"], 1.3e-6 * 10, 1e-5, "colors")
    ins = (m2, cn, cl, op) + ((bg,) if use_bg else ())
    grads = torch.autograd.grad((rc * T(g["v_render_colors"])).sum()
                                + (ra * T(g["v_render_alphas"])).sum(), ins)
    close(grads[0], g["v_means2d"], 5e-3, 5e-3, "v_means2d")
    close(grads[1], g["v_conics"], 1e-3, 1e-3, "v_conics")
    close(grads[2], g["v_colors"], 1e-3, 1e-3, "v_colors")
    close(grads[3], g["v_opacities"], 2e-3, 2e-3, "v_opacities")
    if use_bg:
        close(grads[4], g["v_backgrounds"], 5e-3, 5e-3, "v_backgrounds")
    close(m2.absgrad, g["v_means2d_abs"], 5e-3, 5e-3, "absgrad")


def _garden_scene(n, C, W, H, seed=0, scale=0.02):
    """test_garden.npz is not available on the GPU box: a synthetic scene of the
    same statistics (means in [-2,2]^3 in front of C cameras)."""
    g = torch.Generator().manual_seed(seed)
    means = (torch.rand(n, 3, generator=g) * 4 - 2)
    quats = torch.nn.functional.normalize(torch.randn(n, 4, generator=g), dim=-1)
    scales = torch.rand(n, 3, generator=g) * scale
    opac = torch.rand(n, generator=g)
    vm = torch.eye(4)[None].repeat(C, 1, 1)
    for c in range(C):
        a = 0.4 * c
        vm[c, :3, :3] = torch.tensor([[math.cos(a), 0, math.sin(a)], [0, 1, 0],
                                      [-math.sin(a), 0, math.cos(a)]])
        vm[c, 2, 3] = 5.0
    K = torch.tensor([[0.9 * W, 0, W / 2], [0, 0.9 * W, H / 2], [0, 0, 1]])[None].repeat(C, 1, 1)
    return means, quats, scales, opac, vm, K


@pytest.mark.parametrize("D,tile", [(3, 16), (4, 16), (16, 16), (32, 8), (5, 16)])
def test_raster_vs_oracle_random(D, tile):
    import gsplat_hip
    from oracle import gsplat_oracle as O
    C, N, W, H = 2, 4000, 173, 131
    means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, seed=D, scale=0.05)
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
        means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
    tw, th = math.ceil(W / tile), math.ceil(H / tile)
    _, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, tile, tw, th)
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    gcol = torch.Generator().manual_seed(3)
    cols = torch.rand(C, N, D, generator=gcol).to(DEV)
    ops = opac[None].repeat(C, 1).to(DEV)
    bg = torch.rand(C, D, generator=gcol).to(DEV)
    ins = [x.detach().clone().requires_grad_(True) for x in (m2, cn, cols, ops)]
    rc, ra = gsplat_hip.rasterize_to_pixels(*ins, W, H, tile, off, fids, backgrounds=bg)
    oc, oa, ol = O.raster_fwd(m2.cpu().numpy(), cn.cpu().numpy(), cols.cpu().numpy(),
                              ops.cpu().numpy(), bg.cpu().numpy(), W, H, tile,
                              off.cpu().numpy(), fids.cpu().numpy())
    close_most(ra, oa, 1e-5, 2e-5, "alphas")
    close_most(rc, oc, 1e-5, 2e-5, "colors")
    vrc = torch.randn(rc.shape, generator=gcol).to(DEV)
    vra = torch.randn(ra.shape, generator=gcol).to(DEV)
    grads = torch.autograd.grad((rc * vrc).sum() + (ra * vra).sum(), ins)
    Dp = next(x for x in (1, 2, 3, 4, 8, 16, 32) if x >= D)
    pad = lambda x: np.concatenate([x, np.zeros(x.shape[:-1] + (Dp - D,), np.float32)], -1)
    ref = O.raster_bwd(m2.cpu().numpy(), cn.cpu().numpy(), pad(cols.cpu().numpy()),
                       ops.cpu().numpy(), pad(bg.cpu().numpy()), W, H, tile, off.cpu().numpy(),
                       fids.cpu().numpy(), oa, ol, pad(vrc.cpu().numpy()), vra.cpu().numpy())
    close_most(grads[0], ref[0], 5e-3, 5e-3, "v_means2d", rows=True)
    close_most(grads[1], ref[1], 1e-3, 1e-3, "v_conics", rows=True)
    close_most(grads[2], ref[2][..., :D], 1e-3, 1e-3, "v_colors", rows=True)
    close_most(grads[3], ref[3], 2e-3, 2e-3, "v_opacities")


@pytest.mark.parametrize("chunk", [64, 192])
def test_raster_chunked_backward(chunk):
    """Long tiles split into chunks of `chunk` isects in the backward (state
    saved at the chunk boundaries by the forward) == one work item per tile,
    and == the oracle.  Dense scene: hundreds to thousands of isects per tile,
    many pixels terminating early (T < 1e-4)."""
    import gsplat_hip
    from gsplat_hip import _lib
    from oracle import gsplat_oracle as O
    C, N, W, H, D = 2, 12000, 100, 72, 3
    means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, seed=11, scale=0.12)
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
        means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
    tw, th = math.ceil(W / 16), math.ceil(H / 16)
    _, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th)
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    n_per_tile = np.diff(np.append(off.reshape(-1).cpu().numpy(), ids.numel()))
    assert n_per_tile.max() > 4 * chunk, n_per_tile.max()
    g = torch.Generator().manual_seed(5)
    cols = torch.rand(C, N, D, generator=g).to(DEV)
    ops = opac[None].repeat(C, 1).to(DEV)
    bg = torch.rand(C, D, generator=g).to(DEV)
    vrc = torch.randn(C, H, W, D, generator=g).to(DEV)
    vra = torch.randn(C, H, W, 1, generator=g).to(DEV)

    def run(L):
        # the unsplit forward (its colours are the same up to the chunk sums'
        # rounding); the split forward is tested in test_gpu_raster_dispatch
        _lib.query("gsplat_hip_debug_set_chunk", L)
        split = _lib.query("gsplat_hip_debug_set_fwd_split", 0)
        try:
            ins = [x.detach().clone().requires_grad_(True) for x in (m2, cn, cols, ops)]
            rc, ra = gsplat_hip.rasterize_to_pixels(*ins, W, H, 16, off, fids, backgrounds=bg)
            grads = torch.autograd.grad((rc * vrc).sum() + (ra * vra).sum(), ins,
                                        retain_graph=True)
        finally:
            _lib.query("gsplat_hip_debug_set_chunk", 256)  # the library default
            _lib.query("gsplat_hip_debug_set_fwd_split", split)
        return rc, ra, grads

    rc0, ra0, g0 = run(0)
    rc1, ra1, g1 = run(chunk)
    # the forward sums colour per chunk when chunking: same up to rounding
    assert torch.equal(ra0, ra1)
    torch.testing.assert_close(rc0, rc1, rtol=1e-6, atol=1e-6)
    # Truth: the oracle in float64.  On tiles this long the gradient of a few
    # Gaussians is ill-conditioned (Da = ra * (T gD - rD + ...) cancels, and
    # ra = 1 / (1 - alpha) reaches 500): the fp32 reference algorithm itself
    # (the fp32 oracle) is ~1e-2 off on a few rows there.  Bar: "no worse than
    # the fp32 reference" -- at most max(2, 3x the reference's) rows outside
    # the reference tolerances of float64, and a max error within 2x the
    # reference's max error (+ tolerance).
    lid = _last_ids(rc1)
    outs = {}
    for prec in (np.float64, np.float32):
        args = [x.detach().cpu().numpy().astype(prec) for x in (m2, cn, cols, ops, bg)]
        with O.precision(prec):
            oc, oa, ol = O.raster_fwd(*args, W, H, 16, off.cpu().numpy(), fids.cpu().numpy())
            outs[prec] = (oc, oa) + tuple(O.raster_bwd(
                *args, W, H, 16, off.cpu().numpy(), fids.cpu().numpy(),
                ra1.detach().cpu().numpy().astype(prec), lid, vrc.cpu().numpy().astype(prec),
                vra.cpu().numpy().astype(prec))[:4])
    exact, ref32 = outs[np.float64], outs[np.float32]
    close_most(ra1, exact[1], 1e-5, 2e-5, "alphas")
    close_most(rc1, exact[0], 1e-5, 2e-5, "colors")

    def bad_rows(e, truth, tol):
        bad = e > tol + tol * np.abs(truth)
        return bad.reshape(-1, bad.shape[-1]).any(-1) if bad.ndim > 1 else bad

    for g, how in ((g1, "chunked"), (g0, "whole")):
        for k, (tol, name) in enumerate(((5e-3, "v_means2d"), (1e-3, "v_conics"),
                                         (1e-3, "v_colors"), (2e-3, "v_opacities"))):
            truth = np.asarray(exact[2 + k], np.float64)
            e_ours = np.abs(g[k].detach().cpu().numpy().astype(np.float64) - truth)
            e_ref = np.abs(np.asarray(ref32[2 + k], np.float64) - truth)
            n_ours, n_ref = bad_rows(e_ours, truth, tol).sum(), bad_rows(e_ref, truth, tol).sum()
            assert n_ours <= max(2, 3 * n_ref), (name, how, n_ours, n_ref)
            assert e_ours.max() <= 2 * e_ref.max() + tol, (name, how, e_ours.max(), e_ref.max())


def _last_ids(render_colors):
    """last_ids saved by the rasterize forward (autograd node of its output)."""
    node = render_colors.grad_fn
    return node.saved_tensors[9].cpu().numpy()


def test_raster_tile_masks_skip():
    import gsplat_hip
    C, N, W, H = 1, 500, 64, 48
    means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, scale=0.1)
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
        means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
    _, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, 4, 3)
    off = gsplat_hip.isect_offset_encode(ids, C, 4, 3)
    cols = torch.rand(C, N, 3, device=DEV)
    bg = torch.tensor([[0.1, 0.2, 0.3]], device=DEV)
    masks = torch.zeros(C, 3, 4, dtype=torch.bool, device=DEV)
    masks[0, 1, 2] = True
    rc, ra = gsplat_hip.rasterize_to_pixels(m2, cn, cols, opac[None].to(DEV), W, H, 16, off, fids,
                                            backgrounds=bg, masks=masks)
    rc0, ra0 = gsplat_hip.rasterize_to_pixels(m2, cn, cols, opac[None].to(DEV), W, H, 16, off,
                                              fids, backgrounds=bg)
    blk = (slice(None), slice(16, 32), slice(32, 48))
    assert torch.all(ra[blk] == 0) and torch.allclose(rc[blk], bg.view(1, 1, 1, 3).expand_as(rc[blk]))
    other = torch.ones_like(ra, dtype=torch.bool)
    other[blk] = False
    assert torch.equal(ra[other], ra0[other])


# -------------------------------------------------------- end-to-end M1
# Gradient bars of the end-to-end test, per input: (rtol, atol / max|ref|).
# They are the reference's per-op tolerances of the op that produces each
# gradient last (triton_tests/test_fused_proj.py:159-161 for means / quats /
# scales, test_ras2pix.py:160 for opacities, test_sh.py:35 for the SH
# coefficients, loosened to the rasterizer's 1e-3 bar that feeds them).  The
# achieved errors are written to gpurun_out/e2e_parity_errors.json.
E2E_TOL = {"v_means": (1e-3, 1e-3), "v_quats": (5e-3, 5e-3), "v_scales": (5e-3, 5e-3),
           "v_opacities": (2e-3, 2e-3), "v_sh": (1e-3, 1e-3),
           "v_colors": (1e-3, 1e-3)}  # test_ras2pix.py:160


def _record_errors(name, errs):
    import json
    import os
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "e2e_parity_errors.json")
    try:
        cur = json.load(open(path))
    except (OSError, ValueError):
        cur = {}
    cur[name] = errs
    json.dump(cur, open(path, "w"), indent=1, sort_keys=True)


def _e2e_check(name, g, rc, ra, ins, keys=("v_means", "v_quats", "v_scales", "v_opacities",
                                             "v_sh")):
    errs = {"render_alphas": float(np.abs(ra.detach().cpu().numpy() - g["render_alphas"]).max()),
            "render_colors": float(np.abs(rc.detach().cpu().numpy() - g["render_colors"]).max())}
    # tests/test_rasterization.py:88-89 bars, up to alpha-threshold flips (close_most)
    close_most(ra, g["render_alphas"], 1e-4, 1e-4, "alphas")
    close_most(rc, g["render_colors"], 1e-4, 1e-4, "colors")
    grads = torch.autograd.grad((rc * T(g["v_render_colors"])).sum()
                                + (ra * T(g["v_render_alphas"])).sum(), ins)
    for k, gr in zip(keys, grads):
        ref = g[k]
        scale = max(1e-12, float(np.abs(ref).max()))
        d = np.abs(gr.detach().cpu().numpy().astype(np.float64) - ref)
        errs[k] = {"max_abs": float(d.max()), "max_abs_over_max_ref": float(d.max() / scale),
                   "max_rel_where_big": float((d / np.maximum(np.abs(ref), 1e-3 * scale)).max())}
    _record_errors(name, errs)
    for k, gr in zip(keys, grads):
        ref = g[k]
        rtol, atol = E2E_TOL[k]
        scale = max(1e-12, float(np.abs(ref).max()))
        # a flipped (Gaussian, pixel) pair moves that Gaussian's whole row
        close_most(gr, ref, rtol, atol * scale, k, rows=gr.dim() > 1, out_bound=0.05 * scale)


@pytest.mark.parametrize("name", ["e2e_m1_rgb", "e2e_m1c2_rgbed"])
def test_rasterization_end_to_end_vs_reference(name):
    import gsplat_hip
    g = load_golden(name)
    ins = [T(g[k]).requires_grad_(True) for k in ("means", "quats", "scales", "opacities", "sh")]
    rc, ra, meta = gsplat_hip.rasterization(
        *ins, T(g["viewmats"]), T(g["Ks"]), int(g["width"]), int(g["height"]), sh_degree=3,
        packed=False, render_mode=str(g["render_mode"]), backgrounds=T(g["backgrounds"]))
    assert np.array_equal(meta["radii"].cpu().numpy(), g["radii"])
    assert np.array_equal(meta["isect_ids"].cpu().numpy(), g["isect_ids"])
    assert np.array_equal(meta["flatten_ids"].cpu().numpy(), g["flatten_ids"])
    assert np.array_equal(meta["isect_offsets"].cpu().numpy(), g["isect_offsets"])
    _e2e_check(name, g, rc, ra, ins)


@pytest.mark.parametrize("name", ["e2e_m1_rgb", "e2e_m1c2_rgbed"])
def test_rasterization_packed_vs_reference(name):
    """rasterization(packed=True) against the reference's (dense) goldens: the
    packed pairs are the dense visible entries in (camera, Gaussian) order, so
    radii, the isect keys and -- mapped through (camera_ids, gaussian_ids) --
    the flatten ids equal the reference's exactly; renders and input
    gradients at the same bars as the dense path."""
    import gsplat_hip
    g = load_golden(name)
    ins = [T(g[k]).requires_grad_(True) for k in ("means", "quats", "scales", "opacities", "sh")]
    rc, ra, meta = gsplat_hip.rasterization(
        *ins, T(g["viewmats"]), T(g["Ks"]), int(g["width"]), int(g["height"]), sh_degree=3,
        packed=True, render_mode=str(g["render_mode"]), backgrounds=T(g["backgrounds"]))
    cam = meta["camera_ids"].long().cpu().numpy()
    gid = meta["gaussian_ids"].long().cpu().numpy()
    N = g["radii"].shape[1]
    dense_radii = g["radii"]
    vis = np.argwhere((dense_radii > 0).all(-1) if dense_radii.ndim == 3 else dense_radii > 0)
    assert np.array_equal(np.stack([cam, gid], -1), vis)
    assert np.array_equal(meta["radii"].cpu().numpy(), dense_radii[cam, gid])
    assert np.array_equal(meta["isect_ids"].cpu().numpy(), g["isect_ids"])
    fids = meta["flatten_ids"].long().cpu().numpy()
    assert np.array_equal(cam[fids] * N + gid[fids], g["flatten_ids"])
    assert np.array_equal(meta["isect_offsets"].cpu().numpy(), g["isect_offsets"])
    _e2e_check(name + "_packed", g, rc, ra, ins)


def test_rasterization_antialiased_vs_reference():
    """rasterize_mode="antialiased": opacities multiplied by the projection's
    compensation (gsplat/rendering.py:328,347-351), whose backward runs the
    compensation VJP (fused_projection_bwd.py with calc_compensations)."""
    import gsplat_hip
    g = load_golden("e2e_m1_aa")
    ins = [T(g[k]).requires_grad_(True) for k in ("means", "quats", "scales", "opacities", "sh")]
    rc, ra, meta = gsplat_hip.rasterization(
        *ins, T(g["viewmats"]), T(g["Ks"]), int(g["width"]), int(g["height"]), sh_degree=3,
        packed=False, rasterize_mode="antialiased")
    assert np.array_equal(meta["radii"].cpu().numpy(), g["radii"])
    assert np.array_equal(meta["isect_ids"].cpu().numpy(), g["isect_ids"])
    assert np.array_equal(meta["flatten_ids"].cpu().numpy(), g["flatten_ids"])
    vis = g["radii"] > 0
    # the compensated opacities (test_fused_proj.py:120 bar for compensations)
    close(meta["opacities"].detach().cpu().numpy()[vis], g["opacities_eff"][vis], 5e-4, 1e-3,
          "opacities * compensations")
    _e2e_check("e2e_m1_aa", g, rc, ra, ins)


def test_rasterization_channel_chunks_vs_reference():
    """40 colour channels: rendered in chunks of channel_chunk = 32 (32 + 8,
    gsplat/rendering.py:544-572) with per-channel backgrounds; the alphas of
    the first chunk are returned."""
    import gsplat_hip
    g = load_golden("e2e_m1_d40")
    ins = [T(g[k]).requires_grad_(True)
           for k in ("means", "quats", "scales", "opacities", "colors")]
    rc, ra, meta = gsplat_hip.rasterization(
        *ins, T(g["viewmats"]), T(g["Ks"]), int(g["width"]), int(g["height"]), packed=False,
        backgrounds=T(g["backgrounds"]), channel_chunk=32)
    assert rc.shape[-1] == 40
    assert np.array_equal(meta["radii"].cpu().numpy(), g["radii"])
    assert np.array_equal(meta["isect_ids"].cpu().numpy(), g["isect_ids"])
    assert np.array_equal(meta["flatten_ids"].cpu().numpy(), g["flatten_ids"])
    _e2e_check("e2e_m1_d40", g, rc, ra, ins,
               keys=("v_means", "v_quats", "v_scales", "v_opacities", "v_colors"))


# ------------------------------------------- size-independent properties
def test_full_size_invariants_m2():
    """BASELINE config M2 scale (1M Gaussians, 1080p): properties that hold
    at any size -- sorted keys, offsets = lower_bound, permutation of the
    unsorted isects, alpha in [0, 1), colour = sum of vis*c + T*bg bounds."""
    import gsplat_hip
    C, N, W, H = 1, 1_000_000, 1920, 1080
    means, quats, scales, opac, vm, K = _garden_scene(N, C, W, H, seed=7, scale=0.02)
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(
        means.to(DEV), None, quats.to(DEV), scales.to(DEV), vm.to(DEV), K.to(DEV), W, H)
    tw, th = math.ceil(W / 16), math.ceil(H / 16)
    tpg, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th)
    _, ids_u, fids_u = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th, sort=False)
    assert ids.numel() == int(tpg.sum()) > 1_000_000
    assert torch.all(ids[1:] >= ids[:-1])
    # stable sort <=> (key, unsorted position) pairs sorted
    order = torch.sort(ids_u, stable=True).indices
    assert torch.equal(ids_u[order], ids) and torch.equal(fids_u[order], fids)
    off = gsplat_hip.isect_offset_encode(ids, C, tw, th)
    tiles = torch.arange(C * tw * th, device=DEV, dtype=torch.int64)
    tile_key = (ids >> 32) & ((1 << (tw * th - 1).bit_length()) - 1)
    lb = torch.searchsorted(tile_key.contiguous(), tiles)
    assert torch.equal(off.flatten().long(), lb)
    cols = torch.rand(C, N, 3, device=DEV)
    rc, ra = gsplat_hip.rasterize_to_pixels(m2, cn, cols, opac[None].to(DEV), W, H, 16, off, fids)
    assert torch.isfinite(rc).all() and (ra >= 0).all() and (ra < 1).all()
    assert (rc <= ra + 1e-5).all()  # colours in [0,1] => composite <= alpha


def test_sh_split_coeffs_match_concatenated():
    """(sh0, shN) read in place == the torch.cat'ed [N,K,3] tensor."""
    import gsplat_hip
    torch.manual_seed(1)
    C, N = 2, 999
    sh0 = torch.randn(N, 1, 3, device=DEV, requires_grad=True)
    shN = torch.randn(N, 15, 3, device=DEV, requires_grad=True)
    dirs = torch.randn(C, N, 3, device=DEV, requires_grad=True)
    masks = torch.rand(C, N, device=DEV) > 0.25
    a = gsplat_hip.spherical_harmonics(3, dirs, (sh0.expand(C, -1, -1, -1),
                                                 shN.expand(C, -1, -1, -1)), masks=masks)
    b = gsplat_hip.spherical_harmonics(3, dirs, torch.cat([sh0, shN], 1).expand(C, -1, -1, -1),
                                       masks=masks)
    assert torch.equal(a, b)
    w = torch.randn_like(a)
    ga = torch.autograd.grad((a * w).sum(), (sh0, shN, dirs))
    gb = torch.autograd.grad((b * w).sum(), (sh0, shN, dirs))
    for x, y in zip(ga, gb):
        close(x, y, 1e-6, 1e-6)


@pytest.mark.parametrize("degree,C,split", [(3, 1, True), (3, 2, False), (0, 1, False),
                                            (4, 2, True), (1, 1, False)])
def test_sh_colors_fused_vs_unfused(degree, C, split):
    """rendering.rasterization's colour path fused into one kernel (dirs from
    -R^T t, radii masking, clamp_min(+0.5)) == the reference's torch glue
    around spherical_harmonics (rendering.py:396-406), values and grads."""
    import gsplat_hip
    from gsplat_hip._wrapper import sh_colors
    g = torch.Generator().manual_seed(degree * 10 + C)
    N, K = 3000, (max(degree, 3) + 1) ** 2
    means = (torch.randn(N, 3, generator=g) * 2).to(DEV)
    sh = (torch.randn(N, K, 3, generator=g) * 0.5).to(DEV)
    vm = torch.eye(4).repeat(C, 1, 1)
    for c in range(C):
        q = torch.nn.functional.normalize(torch.randn(4, generator=g), dim=0)
        w, x, y, z = q.tolist()
        vm[c, :3, :3] = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        vm[c, :3, 3] = torch.randn(3, generator=g) * 3
    vm = vm.to(DEV)
    radii = (torch.rand(C, N, generator=g) > 0.3).int().to(DEV) * 5
    vc = torch.randn(C, N, 3, generator=g).to(DEV)

    def unfused(m, s0, sN):
        shs = torch.cat([s0, sN], 1) if split else s0
        dirs = m[None] - torch.inverse(vm)[:, None, :3, 3]
        col = gsplat_hip.spherical_harmonics(degree, dirs, shs.expand(C, -1, -1, -1),
                                             masks=radii > 0)
        return torch.clamp_min(col + 0.5, 0.0)

    def fused(m, s0, sN):
        return sh_colors(degree, m, vm, (s0, sN) if split else s0, radii)

    outs = []
    for fn in (unfused, fused):
        m = means.clone().requires_grad_(True)
        s0 = (sh[:, :1] if split else sh).clone().requires_grad_(True)
        sN = sh[:, 1:].clone().requires_grad_(True) if split else None
        col = fn(m, s0, sN)
        ins = [m, s0] + ([sN] if split else [])
        grads = torch.autograd.grad((col * vc).sum(), ins)
        outs.append((col,) + tuple(grads))
    # campos = -R^T t vs torch.inverse differ by float rounding (R is
    # orthonormal only to ~1e-7); the means gradient at degree 4 amplifies it
    for a, b in zip(outs[0], outs[1]):
        close(b, a, 1e-4, 5e-5)


@pytest.mark.parametrize("degree,C", [(3, 2), (3, 3), (2, 4), (1, 2)])
def test_sh_colors_per_camera_coeffs(degree, C):
    """Per-camera coefficients [C,N,K,3] with K == (degree+1)^2 (the staged
    backward over C*N rows): row i must take camera i // N's centre and
    Gaussian i % N's mean -- against the torch glue of rendering.py:396-406."""
    import gsplat_hip
    from gsplat_hip._wrapper import sh_colors
    g = torch.Generator().manual_seed(100 + degree * 10 + C)
    N, K = 2500, (degree + 1) ** 2
    means = (torch.randn(N, 3, generator=g) * 2).to(DEV)
    sh = (torch.randn(C, N, K, 3, generator=g) * 0.5).to(DEV)
    vm = torch.eye(4).repeat(C, 1, 1)
    for c in range(C):
        q = torch.nn.functional.normalize(torch.randn(4, generator=g), dim=0)
        w, x, y, z = q.tolist()
        vm[c, :3, :3] = torch.tensor([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        vm[c, :3, 3] = torch.randn(3, generator=g) * 3
    vm = vm.to(DEV)
    radii = (torch.rand(C, N, generator=g) > 0.3).int().to(DEV) * 5
    vc = torch.randn(C, N, 3, generator=g).to(DEV)

    def unfused(m, s):
        dirs = m[None] - torch.inverse(vm)[:, None, :3, 3]
        col = gsplat_hip.spherical_harmonics(degree, dirs, s, masks=radii > 0)
        return torch.clamp_min(col + 0.5, 0.0)

    def fused(m, s):
        return sh_colors(degree, m, vm, s, radii)

    outs = []
    for fn in (unfused, fused):
        m = means.clone().requires_grad_(True)
        s = sh.clone().requires_grad_(True)
        col = fn(m, s)
        outs.append((col,) + tuple(torch.autograd.grad((col * vc).sum(), [m, s])))
    for a, b in zip(outs[0], outs[1]):
        close(b, a, 1e-4, 5e-5)


@pytest.mark.parametrize("n_pile", [300, 5000, 20000])
def test_isect_tile_first_long_runs(n_pile):
    """Tiles with very long isect runs: the per-run depth sort switches from
    32 KB LDS (<= 4096) to 128 KB LDS (<= 16384) to a global scratch path."""
    import gsplat_hip
    from gsplat_hip import _wrapper
    g = torch.Generator(device=DEV).manual_seed(n_pile)
    C, ts, tw, th = 2, 16, 6, 5
    N = n_pile + 2000
    m2 = torch.rand(C, N, 2, device=DEV, generator=g) * torch.tensor([tw * ts, th * ts], device=DEV)
    m2[:, :n_pile] = torch.tensor([40.0, 40.0], device=DEV)  # a pile on one tile
    r = (torch.rand(C, N, device=DEV, generator=g) * 6).int()
    r[:, :n_pile] = 3
    d = torch.rand(C, N, device=DEV, generator=g) * 10
    d[:, : n_pile // 3] = 2.5  # ties inside the long run
    d[0, 5:9] = -1.0           # negative depths
    old = _wrapper.ISECT_SORT
    try:
        out = {}
        for mode in ("tile_first", "full"):
            _wrapper.ISECT_SORT = mode
            out[mode] = gsplat_hip.isect_tiles(m2, r, d, ts, tw, th)
    finally:
        _wrapper.ISECT_SORT = old
    for a, b in zip(out["tile_first"], out["full"]):
        assert torch.equal(a, b)


def test_full_size_invariants_m3():
    """BASELINE configs[2] scale (M3: the garden crop tiled 7x7, 5,477,465
    Gaussians, 1920x1080, SH degree 3, the record table above 64 MB):
    size-independent properties -- isect keys sorted, offsets = lower_bound
    of the tile keys, tiles_per_gauss summing to the isect count, the split
    forward at the trainer's M3 divisor (1100) and at a forced 2048-isect
    threshold equal to the unsplit forward up to chunk-product rounding, and
    finite gradients through the split forward's chunk state."""
    import os
    import gsplat_hip
    from gsplat_hip import _lib, _wrapper
    from gsplat_hip.train_step import camera_pool, load_garden_scene
    from test_gpu_parity import close_most
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(root, "tests", "golden", "garden_scene.npz"), scene_grid=7)
    N, W, H = means.shape[0], 1920, 1080
    assert N == 5_477_465
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=1)
    g = torch.Generator().manual_seed(11)
    quats = torch.nn.functional.normalize(torch.randn(N, 4, generator=g), dim=-1)
    scales = torch.rand(N, 3, generator=g) * 0.02
    opac = torch.rand(N, generator=g)
    sh = torch.randn(N, 16, 3, generator=g) * 0.2
    sh[:, 0] = (rgbs - 0.5) / 0.28209479177387814
    ins = [t.to(DEV) for t in (means, quats, scales, opac, sh)]
    vm, K = vm.to(DEV), K.to(DEV)

    # isect invariants at this size
    radii, m2, d, cn, _ = gsplat_hip.fully_fused_projection(ins[0], None, ins[1], ins[2], vm, K,
                                                            W, H)
    tw, th = math.ceil(W / 16), math.ceil(H / 16)
    tpg, ids, fids = gsplat_hip.isect_tiles(m2, radii, d, 16, tw, th)
    assert ids.numel() == int(tpg.sum()) > 3_000_000
    assert torch.all(ids[1:] >= ids[:-1])
    off = gsplat_hip.isect_offset_encode(ids, 1, tw, th)
    tiles = torch.arange(tw * th, device=DEV, dtype=torch.int64)
    tile_key = (ids >> 32) & ((1 << (tw * th - 1).bit_length()) - 1)
    assert torch.equal(off.flatten().long(), torch.searchsorted(tile_key.contiguous(), tiles))
    del ids, fids, tile_key

    def render(split, div=None):
        old = _lib.query("gsplat_hip_debug_set_fwd_split", split)
        try:
            leaves = [x.clone().requires_grad_(True) for x in ins]
            with _wrapper.fwd_split(div):
                rc, ra, meta = gsplat_hip.rasterization(*leaves[:4], leaves[4], vm, K, W, H,
                                                        sh_degree=3, packed=False)
            w = torch.rand(rc.shape, generator=torch.Generator(device=DEV).manual_seed(2),
                           device=DEV)
            (rc * w).sum().backward()
            torch.cuda.synchronize()
            return rc.detach(), ra.detach(), meta, [x.grad for x in leaves]
        finally:
            _lib.query("gsplat_hip_debug_set_fwd_split", old)

    rc0, ra0, m0, g0 = render(0)            # unsplit
    offs = m0["isect_offsets"].flatten().long()
    n = int(m0["flatten_ids"].numel())
    cnt = torch.diff(torch.cat([offs, torch.tensor([n], device=DEV)]))
    thr = max(2048, n // 1100)
    assert int((cnt > 2048).sum()) >= 4, "M3 has heavy tiles"
    for split, div in ((-1, 1100), (2048, None)):  # adaptive at M3's divisor; forced
        if split < 0 and int((cnt > thr).sum()) == 0:
            continue
        rc1, ra1, _, g1 = render(split, div)
        close_most(rc1, rc0, 1e-5, 1e-5, "colors", max_frac=1e-3)
        close_most(ra1, ra0, 1e-5, 1e-5, "alphas", max_frac=1e-3)
        for gg in g1:
            assert torch.isfinite(gg).all()
        for a, b, name in zip(g1, g0, ["means", "quats", "scales", "opacities", "sh"]):
            scale = max(1e-12, float(b.abs().max()))
            close_most(a, b, 1e-3, 1e-4 * scale, name, max_frac=2e-3, rows=True,
                       out_bound=0.05 * scale)
