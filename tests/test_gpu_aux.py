"""GPU parity of the auxiliary kernels (csrc/aux_ops.hip) through the C ABI:
covariance/precision against the reference's torch implementation (goldens),
relocation and the selective Adam against the oracle."""

import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import aux_oracle as A
from test_aux_oracle import binoms

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


@pytest.mark.parametrize("triu", [False, True])
def test_covar_preci_fwd_bwd_vs_reference(triu):
    from gsplat_hip import quat_scale_to_covar_preci
    g = dict(np.load(os.path.join(GOLD, f"covar_preci_triu{int(triu)}.npz")))
    q = torch.tensor(g["quats"], device=DEV, requires_grad=True)
    s = torch.tensor(g["scales"], device=DEV, requires_grad=True)
    cov, pre = quat_scale_to_covar_preci(q, s, triu=triu)
    np.testing.assert_allclose(cov.detach().cpu().numpy(), g["covars"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(pre.detach().cpu().numpy(), g["precis"], rtol=1e-4, atol=1e-3)
    vq, vs = torch.autograd.grad((cov * torch.tensor(g["v_covars"], device=DEV)).sum()
                                 + (pre * torch.tensor(g["v_precis"], device=DEV)).sum(), (q, s))
    # tests/test_basic.py:82-95 tolerances
    np.testing.assert_allclose(vq.cpu().numpy(), g["v_quats"], rtol=1e-1, atol=1e-1)
    np.testing.assert_allclose(vs.cpu().numpy(), g["v_scales"], rtol=1e-1, atol=1e-1)
    scale = np.abs(g["v_scales"]).max()
    assert np.abs(vs.cpu().numpy() - g["v_scales"]).max() <= 1e-3 * scale


def test_covar_only_and_preci_only():
    from gsplat_hip import quat_scale_to_covar_preci
    g = dict(np.load(os.path.join(GOLD, "covar_preci_triu0.npz")))
    q = torch.tensor(g["quats"], device=DEV)
    s = torch.tensor(g["scales"], device=DEV)
    cov, pre = quat_scale_to_covar_preci(q, s, compute_preci=False)
    assert pre is None
    np.testing.assert_allclose(cov.cpu().numpy(), g["covars"], rtol=1e-5, atol=1e-5)
    cov, pre = quat_scale_to_covar_preci(q, s, compute_covar=False, triu=True)
    assert cov is None and pre.shape == (len(q), 6)


def test_relocation_vs_oracle():
    from gsplat_hip import compute_relocation
    rng = np.random.default_rng(2)
    N = 4000
    o = (rng.random(N) * 0.98 + 0.01).astype(np.float32)
    s = rng.random((N, 3)).astype(np.float32)
    r = rng.integers(0, 60, N)
    b = binoms(51)
    ratios = torch.tensor(r, device=DEV)
    no, ns = compute_relocation(torch.tensor(o, device=DEV), torch.tensor(s, device=DEV),
                                ratios, torch.tensor(b, device=DEV))
    rc = np.clip(r, 1, 51)
    assert torch.equal(ratios.cpu(), torch.tensor(rc))  # clamped in place, as the reference
    eo, es = A.relocation(o, s, rc, b)
    np.testing.assert_allclose(no.cpu().numpy(), eo, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(ns.cpu().numpy(), es, rtol=2e-3, atol=1e-6)


@pytest.mark.parametrize("shape", [(1000, 3), (1000,), (1000, 15, 3)])
def test_selective_adam_vs_oracle(shape):
    from gsplat_hip import SelectiveAdam
    rng = np.random.default_rng(len(shape))
    p0 = rng.standard_normal(shape).astype(np.float32)
    param = torch.nn.Parameter(torch.tensor(p0, device=DEV))
    opt = SelectiveAdam([param], eps=1e-15, betas=(0.9, 0.999))
    m = np.zeros_like(p0)
    v = np.zeros_like(p0)
    p = p0
    for it in range(3):
        gr = rng.standard_normal(shape).astype(np.float32)
        vis = rng.random(shape[0]) > 0.3
        param.grad = torch.tensor(gr, device=DEV)
        opt.step(torch.tensor(vis, device=DEV))
        p, m, v = A.adam(p, gr, m, v, vis, opt.param_groups[0]["lr"], 0.9, 0.999, 1e-15)
    np.testing.assert_allclose(param.detach().cpu().numpy(), p, rtol=1e-5, atol=1e-6)
    st = opt.state[param]
    np.testing.assert_allclose(st["exp_avg"].cpu().numpy(), m, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(st["exp_avg_sq"].cpu().numpy(), v, rtol=1e-5, atol=1e-7)
