"""GPU checks of packed mode (§8 f3): the packed projection is the
dense one compacted in (camera, Gaussian) order, its backward (dense and
sparse_grad) sums to the dense backward, and rasterization(packed=True)
renders and differentiates like packed=False."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def scene(N=3000, C=3, W=160, H=120, seed=0):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * torch.tensor([1.0, 0.8, 0.6])
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.08 + 0.005
    opac = torch.rand(N, generator=g)
    sh = torch.randn(N, 16, 3, generator=g) * 0.3
    vms = torch.eye(4).repeat(C, 1, 1)
    for c in range(C):
        vms[c, 0, 3] = 0.3 * c
        vms[c, 1, 3] = -0.1 * c
    K = torch.tensor([[150.0, 0, W / 2], [0, 150.0, H / 2], [0, 0, 1]]).repeat(C, 1, 1)
    return [x.to(DEV) for x in (means, quats, scales, opac, sh, vms, K)] + [W, H]


@pytest.mark.parametrize("C,comp", [(1, False), (3, True)])
def test_packed_fwd_is_dense_compacted(C, comp):
    from gsplat_hip import fully_fused_projection
    means, quats, scales, opac, sh, vms, K, W, H = scene(C=C)
    dense = fully_fused_projection(means, None, quats, scales, vms, K, W, H,
                                   calc_compensations=comp)
    cid, gid, radii, m2, d, cn, cp = fully_fused_projection(
        means, None, quats, scales, vms, K, W, H, packed=True, calc_compensations=comp)
    r, dm2, dd, dcn, dcp = dense
    sel = r > 0
    ec, eg = torch.where(sel)
    assert cid.dtype == torch.int64 and gid.dtype == torch.int64
    assert torch.equal(cid, ec) and torch.equal(gid, eg)
    assert torch.equal(radii, r[sel])
    torch.testing.assert_close(m2, dm2[sel], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(d, dd[sel], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(cn, dcn[sel], rtol=1e-5, atol=1e-5)
    if comp:
        torch.testing.assert_close(cp, dcp[sel], rtol=1e-5, atol=1e-5)
    else:
        assert cp is None


@pytest.mark.parametrize("C,sparse", [(1, False), (3, False), (3, True)])
def test_packed_bwd_matches_dense(C, sparse):
    from gsplat_hip import fully_fused_projection
    means, quats, scales, opac, sh, vms, K, W, H = scene(C=C, seed=1)
    torch.manual_seed(0)

    def grads(packed):
        ins = [x.clone().requires_grad_(True) for x in (means, quats, scales, vms)]
        out = fully_fused_projection(ins[0], None, ins[1], ins[2], ins[3], K, W, H,
                                     packed=packed, sparse_grad=sparse and packed,
                                     calc_compensations=True)
        if packed:
            cid, gid, radii, m2, d, cn, cp = out
        else:
            radii, m2, d, cn, cp = out
        # cotangents drawn densely [C, N, ...], then gathered for the packed pairs
        g = torch.Generator(device=DEV).manual_seed(5)
        N = means.shape[0]
        w = [torch.randn((C, N) + s, device=DEV, generator=g) for s in ((2,), (), (3,), ())]
        if packed:
            w = [wi[cid, gid] for wi in w]
            loss = sum((t * wi).sum() for t, wi in zip((m2, d, cn, cp), w))
        else:  # the kept pairs only
            sel = radii > 0
            loss = sum((t[sel] * wi[sel]).sum() for t, wi in zip((m2, d, cn, cp), w))
        return torch.autograd.grad(loss, ins), out

    (gm_d, gq_d, gs_d, gv_d), _ = grads(False)
    (gm_p, gq_p, gs_p, gv_p), _ = grads(True)
    if sparse:
        assert gm_p.is_sparse
        gm_p, gq_p, gs_p = (x.coalesce().to_dense() for x in (gm_p, gq_p, gs_p))
    for a, b in ((gm_p, gm_d), (gq_p, gq_d), (gs_p, gs_d), (gv_p, gv_d)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()))


@pytest.mark.parametrize("C,mode", [(1, "RGB"), (2, "RGB+D")])
def test_rasterization_packed_matches_dense(C, mode):
    import gsplat_hip
    means, quats, scales, opac, sh, vms, K, W, H = scene(C=C, seed=2)
    res = {}
    for packed in (False, True):
        ins = [x.clone().requires_grad_(True) for x in (means, quats, scales, opac, sh)]
        rc, ra, meta = gsplat_hip.rasterization(*ins, vms, K, W, H, sh_degree=3, packed=packed,
                                                render_mode=mode)
        g = torch.Generator(device=DEV).manual_seed(9)
        loss = (rc * torch.rand(rc.shape, device=DEV, generator=g)).sum() + ra.sum()
        res[packed] = (rc.detach(), ra.detach(), torch.autograd.grad(loss, ins), meta)
    rc0, ra0, g0, m0 = res[False]
    rc1, ra1, g1, m1 = res[True]
    assert m1["camera_ids"] is not None and m1["gaussian_ids"] is not None
    assert m0["isect_ids"].numel() == m1["isect_ids"].numel()
    torch.testing.assert_close(rc1, rc0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ra1, ra0, rtol=1e-5, atol=1e-5)
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4 * float(b.abs().max()))
