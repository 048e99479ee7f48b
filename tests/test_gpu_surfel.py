"""GPU parity of the 2DGS (surfel) path: the HIP kernels (through the C ABI)
against the surfel oracle and the reference's own torch projection goldens.
Tolerances: the reference test's (tests/test_2dgs.py:77-122, 390-396) unless
stated; the rasterizer's ids are exact up to the threshold flips described in
test_gpu_parity.close_most."""

import math

import numpy as np
import pytest
import torch

from oracle import gsplat_oracle as O
from oracle import surfel_oracle as S
from test_gpu_parity import DEV, T, close, close_most
from test_surfel_oracle import _load, surfel_scene

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def _proj_inputs(g):
    return (T(g["means"]), T(g["quats"]), T(g["scales"]), T(g["viewmats"]), T(g["Ks"]),
            int(g["width"]), int(g["height"]))


# -------------------------------------------------------------- projection
@pytest.mark.parametrize("name", ["proj2dgs_testdata.npz", "proj2dgs_random.npz"])
def test_proj2dgs_fwd(name):
    from gsplat_hip import fully_fused_projection_2dgs
    g = _load(name)
    radii, m2, d, rt, nr = fully_fused_projection_2dgs(*_proj_inputs(g))
    o = S.proj2dgs_fwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"],
                       int(g["width"]), int(g["height"]))
    # against the oracle: radii exact up to a ceil() flip, floats to rounding
    close_most(radii, o[0], 0, 0, "radii", max_frac=2e-3, out_bound=1)
    v = (radii.cpu().numpy() > 0) & (o[0] > 0)
    close(m2.cpu().numpy()[v], o[1][v], 1e-4, 1e-4, "means2d")
    close(d, o[2], 1e-5, 1e-6, "depths")
    close(rt.cpu().numpy()[v], o[3][v], 1e-5, 1e-4, "ray_transforms")
    close(nr.cpu().numpy()[v], o[4][v], 1e-5, 1e-6, "normals")
    # against the reference torch implementation (tests/test_2dgs.py:79-85)
    vr = (radii.cpu().numpy() > 0) & (g["radii"] > 0)
    assert np.abs(radii.cpu().numpy() - g["radii"]).max() <= 1
    close(m2.cpu().numpy()[vr], g["means2d"][vr], 1e-4, 1e-4, "means2d vs reference")
    close(rt.cpu().numpy()[vr], g["ray_transforms"][vr], 1e-4, 1e-4, "rt vs reference")
    close(nr.cpu().numpy()[vr], g["normals"][vr], 1e-4, 1e-4, "normals vs reference")


@pytest.mark.parametrize("name", ["proj2dgs_testdata.npz", "proj2dgs_random.npz",
                                  "proj2dgs_random_nomeans2d.npz"])
def test_proj2dgs_bwd(name):
    from gsplat_hip import fully_fused_projection_2dgs
    g = _load(name)
    means, quats, scales, vm, K, W, H = _proj_inputs(g)
    leaves = [x.clone().requires_grad_(True) for x in (means, quats, scales)]
    radii, m2, d, rt, nr = fully_fused_projection_2dgs(*leaves, vm, K, W, H)
    loss = ((m2 * T(g["v_means2d"])).sum() + (d * T(g["v_depths"])).sum()
            + (rt * T(g["v_ray_transforms"])).sum() + (nr * T(g["v_normals"])).sum())
    v_means, v_quats, v_scales = torch.autograd.grad(loss, leaves)
    o_rt = S.proj2dgs_fwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"], W, H)
    om, oq, os_ = S.proj2dgs_bwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"],
                                 radii.cpu().numpy(), o_rt[3], g["v_means2d"], g["v_depths"],
                                 g["v_normals"], g["v_ray_transforms"])
    for a, b, w in ((v_means, om, "v_means"), (v_quats, oq, "v_quats"), (v_scales, os_, "v_scales")):
        close(a, b, 1e-3, 1e-4 * max(1.0, np.abs(b).max()), w)
    assert float(v_scales[:, 2].abs().max()) == 0.0


def test_proj2dgs_viewmats_grad_zero_like_reference():
    """The reference kernel never writes v_viewmats (Projection2DGSFused.cu:319-457)."""
    from gsplat_hip import fully_fused_projection_2dgs
    g = _load("proj2dgs_random.npz")
    means, quats, scales, vm, K, W, H = _proj_inputs(g)
    vm = vm.clone().requires_grad_(True)
    means = means.clone().requires_grad_(True)
    _, m2, d, rt, nr = fully_fused_projection_2dgs(means, quats, scales, vm, K, W, H)
    gv, gm = torch.autograd.grad(rt.sum() + d.sum(), (vm, means))
    assert float(gv.abs().max()) == 0.0 and float(gm.abs().max()) > 0


# ------------------------------------------------------------ rasterizer
def _raster_gpu(sc, masks=None, absgrad=False, D=None):
    from gsplat_hip import rasterize_to_pixels_2dgs
    leaves = {k: T(sc[k]).requires_grad_(True) for k in ("m2", "rt", "colors", "opac", "nr")}
    bg = None if sc["bg"] is None else T(sc["bg"]).requires_grad_(True)
    densify = torch.zeros_like(leaves["m2"], requires_grad=True)
    out = rasterize_to_pixels_2dgs(
        leaves["m2"], leaves["rt"], leaves["colors"], leaves["opac"], leaves["nr"], densify,
        sc["W"], sc["H"], sc["ts"], T(sc["off"]), T(sc["fids"]), backgrounds=bg,
        masks=None if masks is None else T(masks), absgrad=absgrad, distloss=True)
    return leaves, bg, densify, out


def _grads(leaves, extra=()):
    """Leaf gradients in sorted-key order; an absent one (the backward returned
    None: exactly zero, e.g. the normals' without a normal-image gradient)
    as zeros."""
    return [leaves[k].grad if leaves[k].grad is not None else torch.zeros_like(leaves[k])
            for k in sorted(leaves)] + [t.grad if t.grad is not None else torch.zeros_like(t)
                                        for t in extra]


def _oracle_fwd(sc, masks=None):
    return S.raster2dgs_fwd(sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"],
                            masks, sc["W"], sc["H"], sc["ts"], sc["off"], sc["fids"])


@pytest.mark.parametrize("seed,D,bg,C,thin", [(0, 4, True, 1, False), (1, 3, False, 1, False),
                                              (2, 1, True, 2, False), (3, 8, True, 1, False),
                                              (4, 33, False, 1, False), (5, 4, True, 1, True),
                                              (6, 3, False, 2, True)])
def test_raster2dgs_fwd(seed, D, bg, C, thin):
    """thin: needle surfels, many edge-on -- the strip culling's ellipse test
    (surfel_keep) must never drop a contributing record."""
    sc = surfel_scene(seed, N=300, W=70, H=52, D=D, bg=bg, C=C, thin=thin)
    assert len(sc["fids"]) > 200
    _, _, _, (rc, ra, rn, rd, rm) = _raster_gpu(sc)
    oc, oa, on, od, om, ol, omi = _oracle_fwd(sc)
    close_most(rc, oc, 1e-4, 1e-4, "colors", max_frac=5e-3)
    close_most(ra, oa, 1e-4, 1e-4, "alphas", max_frac=5e-3)
    close_most(rn, on, 1e-4, 1e-4, "normals", max_frac=5e-3)
    close_most(rd, od, 1e-3, 1e-3, "distort", max_frac=5e-3)
    close_most(rm, om, 1e-4, 1e-4, "median", max_frac=5e-3)


@pytest.mark.parametrize("seed,D,bg,C,thin,masked", [(0, 4, True, 1, False, False),
                                                     (5, 4, True, 1, True, False),
                                                     (6, 3, False, 2, True, False),
                                                     (2, 1, True, 2, False, True),
                                                     (7, 2, False, 1, False, False)])
def test_raster2dgs_fwd_records_bit_identical(monkeypatch, seed, D, bg, C, thin, masked):
    """The scalar-operand record forward (csrc/surfel.hip fwd2s_kernel,
    GSPLAT_HIP_SURFEL_SREC=1) renders what the LDS-queue forward renders: the
    same per-pixel arithmetic on the same record values, up to the
    compiler's FMA contraction of a few expressions (3.6e-7 seen in one of
    the five outputs); the backward, which reads the forward's outputs and
    last / median ids, agrees to the order of its float atomics."""
    from gsplat_hip import _lib, _wrapper_2dgs
    assert _lib.query("gsplat_hip_rasterize_2dgs_record_floats", D, 16) == 32
    sc = surfel_scene(seed, N=600, W=150, H=100, D=D, bg=bg, C=C, thin=thin)
    masks = (np.random.default_rng(seed).random(sc["off"].shape) > 0.3) if masked else None
    res = []
    for srec in (False, True):
        monkeypatch.setattr(_wrapper_2dgs, "SREC", srec)
        leaves, bgt, densify, out = _raster_gpu(sc, masks=masks)
        w = [torch.linspace(-1, 1, o.numel(), device=DEV).view_as(o) for o in out]
        sum((o * ww).sum() for o, ww in zip(out, w)).backward()
        res.append(([o.detach() for o in out], [leaves[k].grad for k in sorted(leaves)]))
    for a, b, name in zip(res[0][0], res[1][0], ("colors", "alphas", "normals", "distort",
                                                  "median")):
        d = float((a - b).abs().max())
        print(f"{name}: max |diff| {d:.3e}")
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5)
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * float(a.abs().max()))


@pytest.mark.parametrize("masked", [False, True])
def test_raster2dgs_tile_order_changes_nothing(monkeypatch, masked):
    """Heaviest-first dispatch of the tiles (GSPLAT_HIP_SURFEL_ORDER=1): the
    forward's images bit for bit, the backward to the order of its float
    atomics."""
    from gsplat_hip import _wrapper_2dgs
    sc = surfel_scene(3, N=800, W=150, H=100, D=4, bg=True, C=2, thin=True)
    masks = (np.random.default_rng(3).random(sc["off"].shape) > 0.3) if masked else None
    res = []
    for order in (False, True):
        monkeypatch.setattr(_wrapper_2dgs, "ORDER", order)
        leaves, bgt, densify, out = _raster_gpu(sc, masks=masks)
        w = [torch.linspace(-1, 1, o.numel(), device=DEV).view_as(o) for o in out]
        sum((o * ww).sum() for o, ww in zip(out, w)).backward()
        res.append(([o.detach() for o in out], [leaves[k].grad for k in sorted(leaves)]))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b), float((a - b).abs().max())
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * float(a.abs().max()))


def test_raster2dgs_tile_order_above_16384_tiles(monkeypatch):
    """More tiles than one block of the order kernel (2200 x 2100 at 16 px:
    18,216 tiles): the forward writes the dispatch order for every tile (the
    kernel walks 16,384-tile blocks), and the backward, which reuses it,
    sees a complete order -- images bit for bit and gradients as without the
    order (before: no order past 16,384 tiles, and the backward read an
    unwritten one)."""
    from gsplat_hip import _wrapper_2dgs
    sc = surfel_scene(7, N=800, W=2200, H=2100, D=4, bg=True, C=1)
    assert sc["off"].size > 16384
    res = []
    for order in (False, True):
        monkeypatch.setattr(_wrapper_2dgs, "ORDER", order)
        leaves, bgt, densify, out = _raster_gpu(sc)
        w = [torch.linspace(-1, 1, o.numel(), device=DEV).view_as(o) for o in out]
        sum((o * ww).sum() for o, ww in zip(out, w)).backward()
        res.append(([o.detach() for o in out], [leaves[k].grad for k in sorted(leaves)]))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b), float((a - b).abs().max())
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * float(a.abs().max()))


def test_raster2dgs_fwd_masks():
    sc = surfel_scene(5, N=300, W=70, H=52, D=4, bg=True)
    rng = np.random.default_rng(0)
    masks = rng.random(sc["off"].shape) > 0.4
    _, _, _, (rc, ra, rn, rd, rm) = _raster_gpu(sc, masks=masks)
    oc, oa, on, od, om, _, _ = _oracle_fwd(sc, masks=masks)
    close_most(rc, oc, 1e-4, 1e-4, "colors", max_frac=5e-3)
    close_most(ra, oa, 1e-4, 1e-4, "alphas", max_frac=5e-3)


@pytest.mark.parametrize("seed,D,bg,absgrad,thin", [(0, 4, True, False, False),
                                                    (1, 3, False, True, False),
                                                    (2, 1, True, False, False),
                                                    (6, 9, True, True, False),
                                                    (7, 4, True, False, True)])
def test_raster2dgs_bwd(seed, D, bg, absgrad, thin):
    sc = surfel_scene(seed, N=300, W=70, H=52, D=D, bg=bg, thin=thin)
    leaves, bgt, densify, outs = _raster_gpu(sc, absgrad=absgrad)
    rng = np.random.default_rng(seed + 100)
    vs = [rng.standard_normal(o.shape).astype(np.float32) for o in outs]
    loss = sum((o * T(v)).sum() for o, v in zip(outs, vs))
    wrt = list(leaves.values()) + ([bgt] if bgt is not None else []) + [densify]
    grads = torch.autograd.grad(loss, wrt)
    oc, oa, on, od, om, ol, omi = _oracle_fwd(sc)
    ref = S.raster2dgs_bwd(sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"], None,
                           sc["W"], sc["H"], sc["ts"], sc["off"], sc["fids"], oc, oa, ol, omi,
                           *vs, absgrad=absgrad)
    vm, vrt, vcl, vop, vnr, vden, vbg, vab = ref
    names = ["v_means2d", "v_ray_transforms", "v_colors", "v_opacities", "v_normals"]
    for gpu, o, n in zip(grads[:5], (vm, vrt, vcl, vop, vnr), names):
        scale = max(1.0, float(np.abs(o).max()))
        close_most(gpu, o, 1e-3, 1e-3 * scale, n, max_frac=5e-3, rows=True)
    if bg:
        close(grads[5], vbg, 1e-4, 1e-4, "v_backgrounds")
    close_most(grads[-1], vden, 1e-3, 1e-3 * max(1.0, float(np.abs(vden).max())), "v_densify",
               max_frac=5e-3, rows=True)
    if absgrad:
        m2 = leaves["m2"]
        assert m2.absgrad is not None
        close_most(m2.absgrad, vab, 1e-3, 1e-3 * max(1.0, float(np.abs(vab).max())), "absgrad",
                   max_frac=5e-3, rows=True)


@pytest.mark.parametrize("seed,D,bg,absgrad,thin", [(0, 4, True, False, False),
                                                    (1, 3, False, True, False),
                                                    (2, 1, True, False, True)])
def test_raster2dgs_bwd_lean_vs_oracle(seed, D, bg, absgrad, thin):
    """The LEAN backward (csrc/surfel.hip bwd2_kernel<D, ABS, true>): a loss on
    the colours and alphas only -- the normal, distortion and median outputs
    get no gradient (None in the backward), the training step's case -- against
    the oracle's backward with zero gradients for those outputs."""
    sc = surfel_scene(seed, N=300, W=70, H=52, D=D, bg=bg, thin=thin)
    leaves, bgt, densify, outs = _raster_gpu(sc, absgrad=absgrad)
    rng = np.random.default_rng(seed + 200)
    vs = [rng.standard_normal(o.shape).astype(np.float32) for o in outs]
    for i in (2, 3, 4):  # normals, distortion, median: no loss term
        vs[i] = np.zeros_like(vs[i])
    loss = (outs[0] * T(vs[0])).sum() + (outs[1] * T(vs[1])).sum()
    wrt = list(leaves.values()) + ([bgt] if bgt is not None else []) + [densify]
    grads = [torch.zeros_like(t) if g is None else g
             for g, t in zip(torch.autograd.grad(loss, wrt, allow_unused=True), wrt)]
    oc, oa, on, od, om, ol, omi = _oracle_fwd(sc)
    ref = S.raster2dgs_bwd(sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"], None,
                           sc["W"], sc["H"], sc["ts"], sc["off"], sc["fids"], oc, oa, ol, omi,
                           *vs, absgrad=absgrad)
    vm, vrt, vcl, vop, vnr, vden, vbg, vab = ref
    names = ["v_means2d", "v_ray_transforms", "v_colors", "v_opacities", "v_normals"]
    for gpu, o, n in zip(grads[:5], (vm, vrt, vcl, vop, vnr), names):
        scale = max(1.0, float(np.abs(o).max()))
        close_most(gpu, o, 1e-3, 1e-3 * scale, n, max_frac=5e-3, rows=True)
    assert float(grads[4].abs().max()) == 0.0  # v_normals: exactly zero
    if bg:
        close(grads[5], vbg, 1e-4, 1e-4, "v_backgrounds")
    close_most(grads[-1], vden, 1e-3, 1e-3 * max(1.0, float(np.abs(vden).max())), "v_densify",
               max_frac=5e-3, rows=True)
    if absgrad:
        close_most(leaves["m2"].absgrad, vab, 1e-3, 1e-3 * max(1.0, float(np.abs(vab).max())),
                   "absgrad", max_frac=5e-3, rows=True)


def test_raster2dgs_bwd_lean_matches_general():
    """LEAN against the general backward on the same scene: the general one
    runs when the normal / distortion / median outputs get explicit zero
    gradients (the terms LEAN skips are exact zeros), so the two agree to the
    order of their float atomics."""
    sc = surfel_scene(4, N=800, W=150, H=100, D=4, bg=True, C=1, thin=True)
    res = []
    for general in (False, True):
        leaves, bgt, densify, out = _raster_gpu(sc)
        w0 = torch.linspace(-1, 1, out[0].numel(), device=DEV).view_as(out[0])
        loss = (out[0] * w0).sum() + out[1].sum()
        if general:
            loss = loss + sum((o * 0.0).sum() for o in out[2:])
        loss.backward()
        res.append(_grads(leaves, (densify,)))
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("D,masked", [(4, False), (3, True)])
def test_raster2dgs_colors_only_matches_full(D, masked):
    """A colours-only render (ABI 33, `_colors_only`: the training step's)
    forms the full render's colours and alphas (the same arithmetic, up to
    the compiler's FMA contraction in the smaller kernel: 6e-8 seen), returns
    None for the normal / distortion / median images, and its backward (the
    LEAN kernel, no median ids) gives the full render's gradients for a loss
    on the colours and alphas, to the order of the float atomics."""
    from gsplat_hip import rasterize_to_pixels_2dgs
    sc = surfel_scene(8, N=800, W=150, H=100, D=D, bg=True, C=1, thin=True)
    masks = (np.random.default_rng(8).random(sc["off"].shape) > 0.3) if masked else None
    res = []
    for only in (False, True):
        leaves = {k: T(sc[k]).requires_grad_(True) for k in ("m2", "rt", "colors", "opac", "nr")}
        densify = torch.zeros_like(leaves["m2"], requires_grad=True)
        out = rasterize_to_pixels_2dgs(
            leaves["m2"], leaves["rt"], leaves["colors"], leaves["opac"], leaves["nr"], densify,
            sc["W"], sc["H"], sc["ts"], T(sc["off"]), T(sc["fids"]), backgrounds=T(sc["bg"]),
            masks=None if masks is None else T(masks), _colors_only=only)
        if only:
            assert out[2] is None and out[3] is None and out[4] is None
        w0 = torch.linspace(-1, 1, out[0].numel(), device=DEV).view_as(out[0])
        ((out[0] * w0).sum() + out[1].sum()).backward()
        res.append(([out[0].detach(), out[1].detach()], _grads(leaves, (densify,))))
    for a, b in zip(res[0][0], res[1][0]):
        torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-6)
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * max(float(a.abs().max()), 1e-30))


@pytest.mark.parametrize("srec,only", [(True, False), (True, True), (False, False)])
def test_raster2dgs_depth_channel_in_place(monkeypatch, srec, only):
    """The last colour channel read from a separate depths array (ABI 33,
    `_depths`: RGB+D without the concatenated copy) renders what the
    concatenated colours render, bit for bit, and returns that channel's
    gradient to the depths, the rest to the colours (to the atomics' order)."""
    from gsplat_hip import _wrapper_2dgs, rasterize_to_pixels_2dgs
    monkeypatch.setattr(_wrapper_2dgs, "SREC", srec)
    sc = surfel_scene(9, N=800, W=150, H=100, D=4, bg=False, C=1, thin=True)
    res = []
    for split in (False, True):
        leaves = {k: T(sc[k]).requires_grad_(True) for k in ("m2", "rt", "opac", "nr")}
        rgb = T(sc["colors"][..., :3]).requires_grad_(True)
        dep = T(sc["colors"][..., 3]).requires_grad_(True)
        densify = torch.zeros_like(leaves["m2"], requires_grad=True)
        cols = rgb if split else torch.cat([rgb, dep[..., None]], -1)
        out = rasterize_to_pixels_2dgs(
            leaves["m2"], leaves["rt"], cols, leaves["opac"], leaves["nr"], densify,
            sc["W"], sc["H"], sc["ts"], T(sc["off"]), T(sc["fids"]),
            _colors_only=only, _depths=dep if split else None)
        w0 = torch.linspace(-1, 1, out[0].numel(), device=DEV).view_as(out[0])
        loss = (out[0] * w0).sum() + out[1].sum()
        if not only:
            loss = loss + out[2].sum() + 0.5 * out[3].sum() + 0.25 * out[4].sum()
        loss.backward()
        res.append(([o.detach() for o in out if o is not None],
                    _grads(leaves, (rgb, dep, densify))))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b), float((a - b).abs().max())
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5 * max(float(a.abs().max()), 1e-30))


def test_raster2dgs_channel_padding():
    """10 channels are padded to the next compiled count with the depth kept
    last (gsplat/cuda/_wrapper.py:1657-1683); results equal the oracle at 10."""
    sc = surfel_scene(7, N=200, W=48, H=40, D=10, bg=True)
    leaves, bgt, densify, (rc, ra, rn, rd, rm) = _raster_gpu(sc)
    assert rc.shape[-1] == 10
    oc, oa, on, od, om, _, _ = _oracle_fwd(sc)
    # the reference appends the padded background at the end, so the depth
    # channel's background is dropped; surfel_scene's depth background is 0
    close_most(rc, oc, 1e-4, 1e-4, "colors", max_frac=5e-3)
    close_most(rd, od, 1e-3, 1e-3, "distort", max_frac=5e-3)
    g = torch.autograd.grad(rc.sum() + rd.sum(), leaves["colors"])[0]
    assert torch.isfinite(g).all() and g.shape[-1] == 10


def test_raster2dgs_empty():
    from gsplat_hip import rasterize_to_pixels_2dgs
    C, N, W, H = 1, 5, 32, 32
    m2 = torch.zeros(C, N, 2, device=DEV, requires_grad=True)
    rt = torch.zeros(C, N, 3, 3, device=DEV)
    cols = torch.rand(C, N, 3, device=DEV)
    op = torch.rand(C, N, device=DEV)
    nr = torch.zeros(C, N, 3, device=DEV)
    off = torch.zeros(C, 2, 2, dtype=torch.int32, device=DEV)
    fids = torch.zeros(0, dtype=torch.int32, device=DEV)
    bg = torch.rand(C, 3, device=DEV)
    rc, ra, rn, rd, rm = rasterize_to_pixels_2dgs(m2, rt, cols, op, nr, torch.zeros_like(m2), W,
                                                  H, 16, off, fids, backgrounds=bg)
    close(rc, bg[:, None, None, :].expand(C, H, W, 3), 0, 0, "bg only")
    assert float(ra.detach().abs().max()) == 0.0
    (g,) = torch.autograd.grad(rc.sum(), m2)
    assert float(g.abs().max()) == 0.0


# ------------------------------------------------------------- end to end
@pytest.mark.parametrize("mode,sh", [("RGB", None), ("RGB+D", 3), ("RGB+ED", None), ("D", None)])
def test_rasterization_2dgs_e2e(mode, sh):
    from gsplat_hip import rasterization_2dgs
    rng = np.random.default_rng(11)
    N, W, H = 500, 96, 80
    means = (rng.standard_normal((N, 3)) * [0.6, 0.6, 0.3] + [0, 0, 3]).astype(np.float32)
    quats = rng.standard_normal((N, 4)).astype(np.float32)
    scales = (rng.random((N, 3)) * 0.1 + 0.02).astype(np.float32)
    opac = rng.random(N).astype(np.float32)
    if sh is None:
        colors = rng.random((N, 3)).astype(np.float32)
    else:
        colors = (rng.standard_normal((N, (sh + 1) ** 2, 3)) * 0.3).astype(np.float32)
    vm = np.eye(4, dtype=np.float32)[None]
    K = np.array([[90.0, 0, W / 2], [0, 90.0, H / 2], [0, 0, 1]], np.float32)[None]
    leaves = [T(x).requires_grad_(True) for x in (means, quats, scales, opac, colors)]
    bg = T(rng.random((1, 3)).astype(np.float32))
    out = rasterization_2dgs(*leaves, T(vm), T(K), W, H, sh_degree=sh, render_mode=mode,
                             backgrounds=bg if mode != "D" else None, distloss=(mode != "RGB"))
    rc, ra, rn, rnd, rdist, rmed, meta = out
    # oracle composition of the same pipeline
    radii, m2, d, rt, nr = S.proj2dgs_fwd(means, quats, scales, vm, K, W, H)
    assert np.array_equal(meta["radii"].cpu().numpy(), radii)
    tw, th = math.ceil(W / 16), math.ceil(H / 16)
    _, ids, fids = O.isect_tiles(m2, radii, d, 16, tw, th)
    assert np.array_equal(meta["isect_ids"].cpu().numpy(), ids)
    assert np.array_equal(meta["flatten_ids"].cpu().numpy(), fids)
    off = O.isect_offset_encode(ids, 1, tw, th)
    if sh is None:
        cols = colors[None]
    else:
        dirs = means[None] - np.linalg.inv(vm)[:, None, :3, 3]
        cols = np.maximum(O.sh_fwd(sh, dirs, colors[None], masks=radii > 0) + 0.5, 0)
    bgo = bg.cpu().numpy()
    if mode in ("RGB+D", "RGB+ED"):
        cols = np.concatenate([cols, d[..., None]], -1)
        bgo = np.concatenate([bgo, np.zeros((1, 1), np.float32)], -1)
    elif mode == "D":
        cols, bgo = d[..., None], None
    oc, oa, on, od, om, _, _ = S.raster2dgs_fwd(m2, rt, cols, opac[None], nr, bgo, None, W, H, 16,
                                                off, fids)
    if mode in ("ED", "RGB+ED"):
        oc = np.concatenate([oc[..., :-1], oc[..., -1:] / np.maximum(oa, 1e-10)], -1)
    close_most(rc, oc, 1e-4, 1e-4, "colors", max_frac=5e-3)
    close_most(ra, oa, 1e-4, 1e-4, "alphas", max_frac=5e-3)
    close_most(rn, on, 1e-4, 1e-4, "normals (camera = world here)", max_frac=5e-3)
    if mode in ("RGB+D", "RGB+ED"):
        assert rnd is not None and rnd.shape == (H, W, 3)
    loss = rc.sum() + ra.sum() + rn.sum() + rdist.sum()
    loss.backward()
    for i, x in enumerate(leaves):
        if mode == "D" and i == 4:  # colours are not rendered in depth mode
            assert x.grad is None
            continue
        assert x.grad is not None and torch.isfinite(x.grad).all()
    assert meta["gradient_2dgs"].grad is not None
    assert float(meta["gradient_2dgs"].grad.abs().sum()) > 0


@pytest.mark.parametrize("z_depth,C", [(True, 1), (False, 2)])
def test_depth_to_normal_matches_torch_formula(z_depth, C):
    """HIP depth_to_normal (forward) against the reference formula
    (gsplat/utils.py:201-224) in torch, and its gradient."""
    from gsplat_hip.rendering import _depth_to_normal_torch, depth_to_normal
    g = torch.Generator(device=DEV).manual_seed(3)
    H, W = 37, 53
    d = (2.0 + torch.rand(C, H, W, 1, device=DEV, generator=g)).requires_grad_(True)
    vm = torch.eye(4, device=DEV).repeat(C, 1, 1)
    vm[:, :3, 3] = torch.randn(C, 3, device=DEV, generator=g) * 0.3
    c2w = torch.linalg.inv(vm)
    K = torch.tensor([[60.0, 0, W / 2], [0, 55.0, H / 2], [0, 0, 1]], device=DEV).repeat(C, 1, 1)
    a = depth_to_normal(d, c2w, K, z_depth=z_depth)
    b = _depth_to_normal_torch(d, c2w, K, z_depth=z_depth)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    w = torch.randn_like(b)
    ga, = torch.autograd.grad((a * w).sum(), d)
    gb, = torch.autograd.grad((b * w).sum(), d)
    torch.testing.assert_close(ga, gb, rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------- packed
@pytest.mark.parametrize("name", ["proj2dgs_testdata.npz", "proj2dgs_random.npz"])
def test_proj2dgs_packed_fwd_vs_reference(name):
    """Packed projection (Projection2DGSPacked.cu) against the reference torch
    goldens: the kept (camera, surfel) pairs in (camera, surfel) order, each
    with the dense golden's values (a ceil() flip of radii may add or drop a
    pair at the visibility edge)."""
    from gsplat_hip import fully_fused_projection_2dgs
    g = _load(name)
    cid, gid, radii, m2, d, rt, nr = fully_fused_projection_2dgs(*_proj_inputs(g), packed=True)
    dense = fully_fused_projection_2dgs(*_proj_inputs(g), packed=False)
    keep = dense[0].cpu().numpy() > 0
    c_ref, n_ref = np.nonzero(keep)  # row-major: camera, then surfel
    assert np.array_equal(cid.cpu().numpy(), c_ref) and np.array_equal(gid.cpu().numpy(), n_ref)
    # the packed kernel recomputes what the dense one does (up to FMA
    # contraction in a separately compiled kernel)
    assert torch.equal(radii, dense[0][keep])
    for p, dn, w in zip((m2, d, rt, nr), dense[1:], ("means2d", "depths", "rt", "normals")):
        close(p, dn[keep], 1e-5, 1e-4, w + " packed vs dense")
    vr = g["radii"][c_ref, n_ref] > 0
    assert np.abs(radii.cpu().numpy() - g["radii"][c_ref, n_ref]).max() <= 1
    close(m2.cpu().numpy()[vr], g["means2d"][c_ref, n_ref][vr], 1e-4, 1e-4, "means2d vs reference")
    close(rt.cpu().numpy()[vr], g["ray_transforms"][c_ref, n_ref][vr], 1e-4, 1e-4, "rt vs reference")
    close(nr.cpu().numpy()[vr], g["normals"][c_ref, n_ref][vr], 1e-4, 1e-4,
          "normals vs reference")


@pytest.mark.parametrize("name,sparse", [("proj2dgs_testdata.npz", False),
                                         ("proj2dgs_random.npz", False),
                                         ("proj2dgs_random.npz", True)])
def test_proj2dgs_packed_bwd_vs_oracle(name, sparse):
    """Packed backward (dense atomics or sparse COO rows) against the oracle
    VJP of the same cotangents scattered onto the dense [C, N] layout."""
    from gsplat_hip import fully_fused_projection_2dgs
    g = _load(name)
    means, quats, scales, vm, K, W, H = _proj_inputs(g)
    leaves = [x.clone().requires_grad_(True) for x in (means, quats, scales)]
    cid, gid, radii, m2, d, rt, nr = fully_fused_projection_2dgs(*leaves, vm, K, W, H,
                                                                 packed=True, sparse_grad=sparse)
    c_i, n_i = cid.cpu().numpy(), gid.cpu().numpy()
    sel = lambda a: T(np.ascontiguousarray(a[c_i, n_i]))  # noqa: E731
    loss = ((m2 * sel(g["v_means2d"])).sum() + (d * sel(g["v_depths"])).sum()
            + (rt * sel(g["v_ray_transforms"])).sum() + (nr * sel(g["v_normals"])).sum())
    grads = torch.autograd.grad(loss, leaves)
    if sparse:
        assert all(x.is_sparse for x in grads)
        grads = [x.to_dense() for x in grads]
    keep = np.zeros(g["radii"].shape, bool)
    keep[c_i, n_i] = True
    zero = lambda a: np.where(keep.reshape(keep.shape + (1,) * (a.ndim - 2)), a, 0)  # noqa: E731
    o_rt = S.proj2dgs_fwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"], W, H)
    radii_dense = np.where(keep, np.maximum(o_rt[0], 1), 0).astype(np.int32)
    om, oq, os_ = S.proj2dgs_bwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"],
                                 radii_dense, o_rt[3], zero(g["v_means2d"]), zero(g["v_depths"]),
                                 zero(g["v_normals"]), zero(g["v_ray_transforms"]))
    for a, b, w in zip(grads, (om, oq, os_), ("v_means", "v_quats", "v_scales")):
        close(a, b, 1e-3, 1e-4 * max(1.0, np.abs(b).max()), w)


@pytest.mark.parametrize("mode,sh", [("RGB", None), ("RGB+D", 3)])
def test_rasterization_2dgs_packed_matches_dense(mode, sh):
    """rasterization_2dgs(packed=True) (gsplat/rendering.py:1188-1236) renders
    the same images as the dense path (same per-pixel records in the same
    order) and gives the same parameter gradients; the dense path is pinned
    against the oracle by test_rasterization_2dgs_e2e."""
    from gsplat_hip import rasterization_2dgs
    rng = np.random.default_rng(12)
    N, W, H, C = 600, 96, 80, 2
    means = (rng.standard_normal((N, 3)) * [0.6, 0.6, 0.3] + [0, 0, 3]).astype(np.float32)
    quats = rng.standard_normal((N, 4)).astype(np.float32)
    scales = (rng.random((N, 3)) * 0.1 + 0.02).astype(np.float32)
    opac = rng.random(N).astype(np.float32)
    colors = (rng.random((N, 3)).astype(np.float32) if sh is None else
              (rng.standard_normal((N, (sh + 1) ** 2, 3)) * 0.3).astype(np.float32))
    vm = np.tile(np.eye(4, dtype=np.float32), (C, 1, 1))
    vm[1, 0, 3] = 0.2
    K = np.tile(np.array([[90.0, 0, W / 2], [0, 90.0, H / 2], [0, 0, 1]], np.float32), (C, 1, 1))
    outs, grads = [], []
    for packed in (False, True):
        leaves = [T(x).requires_grad_(True) for x in (means, quats, scales, opac, colors)]
        o = rasterization_2dgs(*leaves, T(vm), T(K), W, H, sh_degree=sh, render_mode=mode,
                               packed=packed, distloss=mode != "RGB")
        rc, ra, rn, rnd, rdist, rmed, meta = o
        (rc.sum() + ra.sum() + rn.sum() + rdist.sum()).backward()
        outs.append((rc, ra, rn, rdist, rmed))
        grads.append([x.grad for x in leaves])
        if packed:
            assert meta["camera_ids"] is not None and meta["gaussian_ids"] is not None
    for a, b, n in zip(outs[0], outs[1], ("colors", "alphas", "normals", "distort", "median")):
        close(b, a, 1e-5, 1e-5, n)
    for a, b, n in zip(grads[0], grads[1], ("means", "quats", "scales", "opacities", "colors")):
        close(b, a, 1e-4, 1e-5 * max(1.0, float(a.abs().max())), n)


@pytest.mark.parametrize("thin,dense", [(False, False), (True, False), (False, True)])
def test_capped_surfel_tile_culling_changes_no_render(thin, dense):
    """The captured 2DGS step's isect (gsplat_hip_isect_write_sorted_capped_surfel,
    rasterization_2dgs(_isect_capacity=..., _colors_only=True)): surfels whose
    tile rectangle spans more than 16 supertiles get isects only in the tiles
    their image can reach.  The scene has large and edge-on (thin) surfels
    whose rectangles cover most of the image; fewer isects are written than
    the rectangles hold, and the render -- colours and alphas -- equals the
    uncapped colours-only render bit for bit (the rasterizer culls exactly
    those isects on every strip); the gradients agree at the float atomics'
    run-to-run spread.  `dense`: most surfels large at 1080p -- over a
    million (supertile, surfel) pairs, more than one sweep of the culling
    kernel's grid-stride loop (2048 x 256 lanes)."""
    from gsplat_hip import rasterization_2dgs, rendering
    rng = np.random.default_rng(21)
    N, W, H = (8000, 1920, 1080) if dense else (3000, 1280, 720)
    means = (rng.standard_normal((N, 3)) * [1.2, 0.8, 0.4] + [0, 0, 3]).astype(np.float32)
    quats = rng.standard_normal((N, 4)).astype(np.float32)
    scales = (rng.random((N, 3)) * 0.05 + 0.005).astype(np.float32)
    big = rng.random(N) < (0.6 if dense else 0.03)  # large: rectangles over many supertiles
    scales[big, :2] *= 20.0
    if thin:  # needles seen edge-on: long thin images across the frame
        scales[:, 1] = rng.uniform(0.0005, 0.002, N)
    opac = rng.random(N).astype(np.float32)
    sh = (rng.standard_normal((N, 16, 3)) * 0.3).astype(np.float32)
    vm = np.eye(4, dtype=np.float32)[None]
    K = np.array([[900.0, 0, W / 2], [0, 900.0, H / 2], [0, 0, 1]], np.float32)[None]
    res = []
    for capped in (False, True, False):
        leaves = [T(x).requires_grad_(True) for x in (means, quats, scales, opac, sh)]
        kw = dict(_isect_capacity=(48 << 20) if dense else (4 << 20)) if capped else {}
        rc, ra, _, _, _, _, meta = rasterization_2dgs(
            *leaves[:4], leaves[4], T(vm), T(K), W, H, sh_degree=3, render_mode="RGB+D",
            _colors_only=True, **kw)
        w = torch.linspace(-1, 1, rc.numel(), device=DEV).view_as(rc)
        (rc * w).sum().backward()
        torch.cuda.synchronize()
        res.append((rc.detach(), ra.detach(), [x.grad for x in leaves], meta))
    (rc0, ra0, g0, m0), (rc1, ra1, g1, m1), (_, _, g0b, _) = res
    counts = m1["isect_counts"].cpu().numpy()
    n_rect = int(m0["flatten_ids"].numel())
    assert counts[2] == 0 and counts[3] == n_rect, (counts, n_rect)
    assert counts[0] < n_rect, "no isect culled: the scene has no large surfel"
    print(f"isects written {counts[0]} of {n_rect} ({counts[0] / n_rect:.3f})")
    assert rendering.TILE_CULL
    assert torch.equal(rc0, rc1) and torch.equal(ra0, ra1)
    for a, a2, b, name in zip(g0, g0b, g1, ["means", "quats", "scales", "opac", "sh"]):
        scale = float(a.abs().max())
        spread = float((a2 - a).abs().max())
        err = float((b - a).abs().max())
        assert err <= max(4.0 * spread, 1e-5 * scale) + 1e-12, (name, err, spread, scale)
