"""CPU checks of the auxiliary-kernel oracle (oracle/aux_oracle.py)."""

import math
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import aux_oracle as A

GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.parametrize("triu", [False, True])
def test_covar_preci_vs_reference_torch(triu):
    g = dict(np.load(os.path.join(GOLD, f"covar_preci_triu{int(triu)}.npz")))
    cov, pre = A.covar_preci(g["quats"], g["scales"], triu=triu)
    # tests/test_basic.py:69-70 tolerances (torch.testing defaults for fp32)
    np.testing.assert_allclose(cov, g["covars"], rtol=1.3e-6, atol=1e-5)
    np.testing.assert_allclose(pre, g["precis"], rtol=1e-4, atol=1e-3)


def binoms(n_max=51):
    b = np.zeros((n_max, n_max), np.float32)
    for n in range(n_max):
        for k in range(n + 1):
            b[n, k] = math.comb(n, k)
    return b


def test_relocation_opacity_identity():
    """MCMC Eq. 8: n copies with opacity o' composite to the old opacity o."""
    rng = np.random.default_rng(0)
    o = rng.random(64).astype(np.float32) * 0.98 + 0.01
    s = rng.random((64, 3)).astype(np.float32)
    n = rng.integers(1, 12, 64)
    no, ns = A.relocation(o, s, n, binoms())
    np.testing.assert_allclose(1 - (1 - no.astype(np.float64)) ** n, o, rtol=1e-5, atol=1e-6)
    assert np.all(ns[n == 1] == s[n == 1]) or np.allclose(ns[n == 1], s[n == 1], rtol=1e-6)


def test_adam_oracle_vs_torch_formula():
    rng = np.random.default_rng(1)
    p, g, m, v = (rng.standard_normal((40, 5, 3)).astype(np.float32) for _ in range(4))
    v = np.abs(v)
    valid = rng.random(40) > 0.5
    P, M, V = A.adam(p, g, m, v, valid, 1e-2, 0.9, 0.999, 1e-15)
    tp, tg, tm, tv = (torch.tensor(x) for x in (p, g, m, v))
    m2 = 0.9 * tm + 0.1 * tg
    v2 = 0.999 * tv + 0.001 * tg * tg
    p2 = tp - 1e-2 * m2 / (v2.sqrt() + 1e-15)
    sel = torch.tensor(valid)[:, None, None]
    np.testing.assert_allclose(P, torch.where(sel, p2, tp).numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(M, torch.where(sel, m2, tm).numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(V, torch.where(sel, v2, tv).numpy(), rtol=1e-6, atol=1e-7)
