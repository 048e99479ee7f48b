"""CPU checks of the 2DGS (surfel) oracle.

* projection forward/backward against the reference's own torch
  implementation (golden vectors from tests/golden/make_golden_2dgs.py), at
  the reference test's tolerances (tests/test_2dgs.py:77-122);
* rasterization: no reference outputs can be produced here (the
  reference's torch rasterizer needs the CUDA extension and nerfacc), so the
  oracle's forward is compared with an independent torch restatement of
  RasterizeToPixels2DGSFwd.cu, and the oracle's hand-derived backward
  (RasterizeToPixels2DGSBwd.cu) with torch autograd of that restatement.
"""

import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import gsplat_oracle as O
from oracle import surfel_oracle as S

GOLD = os.path.join(ROOT, "tests", "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLD, name)))


@pytest.mark.parametrize("name", ["proj2dgs_testdata.npz", "proj2dgs_random.npz"])
def test_proj2dgs_fwd_golden(name):
    g = _load(name)
    radii, m2, d, rt, nr = S.proj2dgs_fwd(g["means"], g["quats"], g["scales"], g["viewmats"],
                                          g["Ks"], int(g["width"]), int(g["height"]))
    assert np.abs(radii - g["radii"]).max() <= 1
    v = (radii > 0) & (g["radii"] > 0)
    assert v.sum() > 0.9 * v.size
    np.testing.assert_allclose(m2[v], g["means2d"][v], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(d[v], g["depths"][v], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(rt[v], g["ray_transforms"][v], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(nr[v], g["normals"][v], rtol=1e-4, atol=1e-4)


def _proj_bwd(g):
    args = (g["viewmats"], g["Ks"], int(g["width"]), int(g["height"]))
    radii, _, _, rt, _ = S.proj2dgs_fwd(g["means"], g["quats"], g["scales"], *args)
    return S.proj2dgs_bwd(g["means"], g["quats"], g["scales"], g["viewmats"], g["Ks"], radii, rt,
                          g["v_means2d"], g["v_depths"], g["v_normals"], g["v_ray_transforms"])


def test_proj2dgs_bwd_golden_reference_scene():
    """The reference test's scene and tolerances (tests/test_2dgs.py:117-122)."""
    g = _load("proj2dgs_testdata.npz")
    vm, vq, vs = _proj_bwd(g)
    np.testing.assert_allclose(vq, g["v_quats"], rtol=2e-1, atol=1e-2)
    np.testing.assert_allclose(vs[..., :2], g["v_scales"][..., :2], rtol=1e-1, atol=2e-1)
    np.testing.assert_allclose(vm, g["v_means"], rtol=1e-2, atol=6e-2)


def test_proj2dgs_bwd_golden_random():
    """Random scene: the CUDA means2d VJP drops the cross terms of the AABB
    formula (Projection2DGS.cuh:25-65), so it is not autograd's exact
    gradient; the reference test's tolerances hold relative to the gradient
    scale."""
    g = _load("proj2dgs_random.npz")
    vm, vq, vs = _proj_bwd(g)
    for a, b in ((vq, g["v_quats"]), (vs[..., :2], g["v_scales"][..., :2]), (vm, g["v_means"])):
        scale = np.abs(b).max()
        np.testing.assert_allclose(a, b, rtol=2e-1, atol=2e-2 * scale)
        assert np.abs(a - b).mean() <= 2e-3 * scale


def test_proj2dgs_bwd_golden_exact_part():
    """v_means2d = 0: the remaining VJP is exact -- tight agreement with autograd."""
    g = _load("proj2dgs_random_nomeans2d.npz")
    vm, vq, vs = _proj_bwd(g)
    for a, b in ((vq, g["v_quats"]), (vs[..., :2], g["v_scales"][..., :2]), (vm, g["v_means"])):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4 * np.abs(b).max())


# ---------------------------------------------------------------- raster ---
def surfel_scene(seed=0, N=60, W=40, H=36, D=4, bg=True, C=1, thin=False):
    rng = np.random.default_rng(seed)
    means = (rng.standard_normal((N, 3)) * [0.5, 0.5, 0.3] + [0, 0, 3]).astype(np.float32)
    quats = rng.standard_normal((N, 4)).astype(np.float32)
    scales = (rng.random((N, 3)) * 0.25 + 0.05).astype(np.float32)
    if thin:  # needle-like surfels (one axis 100x shorter), many seen edge-on
        scales[:, 0] = rng.uniform(0.2, 0.8, N)
        scales[:, 1] = rng.uniform(0.001, 0.008, N)
    vm = np.tile(np.eye(4, dtype=np.float32), (C, 1, 1))
    vm[:, 0, 3] = np.arange(C) * 0.1
    K = np.tile(np.array([[60.0, 0, W / 2], [0, 60.0, H / 2], [0, 0, 1]], np.float32), (C, 1, 1))
    radii, m2, depths, rt, nr = S.proj2dgs_fwd(means, quats, scales, vm, K, W, H)
    ts = 16
    tw, th = math.ceil(W / ts), math.ceil(H / ts)
    _, ids, fids = O.isect_tiles(m2, radii, depths, ts, tw, th)
    off = O.isect_offset_encode(ids, C, tw, th)
    colors = rng.random((C, N, D)).astype(np.float32)
    colors[..., -1] = depths
    opac = (rng.random((C, N)) * 0.9 + 0.05).astype(np.float32)
    bgs = rng.random((C, D)).astype(np.float32) if bg else None
    if bg:
        # rasterization_2dgs appends a zero background for the depth channel
        # (gsplat/rendering.py:1250-1256); the reference backward reads the
        # depth sum from render_colors, which is exact only in that case
        bgs[:, -1] = 0.0
    return dict(m2=m2, rt=rt, colors=colors, opac=opac, nr=nr, bg=bgs, W=W, H=H, ts=ts,
                off=off, fids=fids, radii=radii)


def torch_raster2dgs(m2, rt, colors, opac, nr, bg, W, H, ts, off, fids):
    """Independent torch restatement of RasterizeToPixels2DGSFwd.cu:229-450
    (sequential over a tile's isects, vectorised over its pixels)."""
    C, th, tw = off.shape
    D = colors.shape[-1]
    flat = np.asarray(off).reshape(-1)
    ends = np.append(flat[1:], len(fids))
    m2f, rtf = m2.reshape(-1, 2), rt.reshape(-1, 9)
    clf, opf, nrf = colors.reshape(-1, D), opac.reshape(-1), nr.reshape(-1, 3)
    outs = {k: torch.zeros((C, H, W) + s) for k, s in
            (("c", (D,)), ("a", (1,)), ("n", (3,)), ("d", (1,)), ("m", (1,)))}
    res = {k: [] for k in outs}
    for t in range(C * th * tw):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        ys, xs = np.meshgrid(np.arange(ts) + ty * ts, np.arange(ts) + tx * ts, indexing="ij")
        ys, xs = ys.reshape(-1), xs.reshape(-1)
        ins = (ys < H) & (xs < W)
        ys, xs = ys[ins], xs[ins]
        px = torch.tensor(xs, dtype=torch.float32) + 0.5
        py = torch.tensor(ys, dtype=torch.float32) + 0.5
        P = len(ys)
        T = torch.ones(P)
        done = torch.zeros(P, dtype=torch.bool)
        col, nrm = torch.zeros(P, D), torch.zeros(P, 3)
        dist, avd, med = torch.zeros(P), torch.zeros(P), torch.zeros(P)
        for j in range(flat[t], ends[t]):
            g = int(fids[j])
            m = rtf[g]
            hu = px[:, None] * m[6:9] - m[0:3]
            hv = py[:, None] * m[6:9] - m[3:6]
            rc = torch.cross(hu, hv, dim=-1)
            s = rc[:, :2] / rc[:, 2:3]
            g3 = (s * s).sum(-1)
            d = m2f[g][None] - torch.stack([px, py], -1)
            g2 = 2.0 * (d * d).sum(-1)
            sig = 0.5 * torch.minimum(g3, g2)
            alpha = torch.clamp_max(opf[g] * torch.exp(-sig), 0.999)
            ok = (rc[:, 2] != 0) & ~(sig < 0) & ~(alpha < 1.0 / 255.0) & ~done
            nT = T * (1.0 - alpha)
            stop = ok & (nT <= 1e-4)
            done = done | stop
            act = ok & ~stop
            vis = torch.where(act, alpha * T, torch.zeros(()))
            col = col + vis[:, None] * clf[g][None]
            nrm = nrm + vis[:, None] * nrf[g][None]
            depth = clf[g][D - 1]
            dist = torch.where(act, dist + 2.0 * (vis * depth * (1.0 - T) - vis * avd), dist)
            avd = torch.where(act, avd + vis * depth, avd)
            med = torch.where(act & (T > 0.5), depth.expand(P), med)
            T = torch.where(act, nT, T)
        if bg is not None:
            col = col + T[:, None] * bg[c][None]
        res["c"].append((c, ys, xs, col))
        res["a"].append((c, ys, xs, (1.0 - T)[:, None]))
        res["n"].append((c, ys, xs, nrm))
        res["d"].append((c, ys, xs, dist[:, None]))
        res["m"].append((c, ys, xs, med[:, None]))
    final = {}
    for k, parts in res.items():
        o = outs[k].clone()
        for c, ys, xs, v in parts:
            o = o.index_put((torch.full((len(ys),), c), torch.tensor(ys), torch.tensor(xs)), v)
        final[k] = o
    return final


@pytest.mark.parametrize("seed,bg", [(0, True), (1, False)])
def test_raster2dgs_oracle_fwd_matches_torch(seed, bg):
    sc = surfel_scene(seed, bg=bg)
    oc, oa, on, od, om, ol, omi = S.raster2dgs_fwd(
        sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"], None, sc["W"], sc["H"],
        sc["ts"], sc["off"], sc["fids"])
    tt = torch_raster2dgs(*(torch.tensor(sc[k]) if isinstance(sc[k], np.ndarray) and k != "off"
                            and k != "fids" else sc[k]
                            for k in ("m2", "rt", "colors", "opac", "nr", "bg", "W", "H", "ts",
                                      "off", "fids")))
    assert len(sc["fids"]) > 100
    for o, k in ((oc, "c"), (oa, "a"), (on, "n"), (od, "d"), (om, "m")):
        np.testing.assert_allclose(o, tt[k].numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("seed,bg,absgrad", [(0, True, False), (2, False, True)])
def test_raster2dgs_oracle_bwd_matches_autograd(seed, bg, absgrad):
    sc = surfel_scene(seed, bg=bg)
    args = ("m2", "rt", "colors", "opac", "nr", "bg")
    leaves = {k: torch.tensor(sc[k], requires_grad=True) for k in args if sc[k] is not None}
    tt = torch_raster2dgs(*(leaves.get(k) for k in args), sc["W"], sc["H"], sc["ts"], sc["off"],
                          sc["fids"])
    rng = np.random.default_rng(seed + 10)
    vs = {k: rng.standard_normal(tt[k].shape).astype(np.float32) for k in tt}
    loss = sum((tt[k] * torch.tensor(vs[k])).sum() for k in tt)
    grads = dict(zip(leaves, torch.autograd.grad(loss, list(leaves.values()))))

    oc, oa, on, od, om, ol, omi = S.raster2dgs_fwd(
        sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"], None, sc["W"], sc["H"],
        sc["ts"], sc["off"], sc["fids"])
    vm, vrt, vcl, vop, vnr, vden, vbg, vab = S.raster2dgs_bwd(
        sc["m2"], sc["rt"], sc["colors"], sc["opac"], sc["nr"], sc["bg"], None, sc["W"], sc["H"],
        sc["ts"], sc["off"], sc["fids"], oc, oa, ol, omi, vs["c"], vs["a"], vs["n"], vs["d"],
        vs["m"], absgrad=absgrad)
    tol = dict(rtol=2e-3, atol=2e-3)
    np.testing.assert_allclose(vm, grads["m2"].numpy(), **tol)
    np.testing.assert_allclose(vrt, grads["rt"].numpy(), **tol)
    np.testing.assert_allclose(vcl, grads["colors"].numpy(), **tol)
    np.testing.assert_allclose(vop, grads["opac"].numpy(), **tol)
    np.testing.assert_allclose(vnr, grads["nr"].numpy(), **tol)
    if bg:
        np.testing.assert_allclose(vbg, grads["bg"].numpy(), **tol)
    if absgrad:
        assert (vab >= np.abs(vm) - 1e-6).all()
    np.testing.assert_allclose(vden[..., 0], vrt[..., 0, 2] * sc["rt"][..., 2, 2], rtol=1e-6)
