"""GPU: DefaultStrategy's refine step on the HIP backend (gsplat_hip.densify,
csrc/strategy.hip) against goldens produced by the reference's own
_grow_gs / _prune_gs / reset_opa with torch.optim.Adam
(tests/golden/make_golden_strategy.py), fed the same split noise.

Bars as tests/test_strategy_oracle.py: counts, row order, copied values and
the optimizer moments exact; split children's means / log-scales (and
revised-opacity logits) within a few fp32 ulps."""

import numpy as np
import pytest
import torch

from conftest import load_golden
from test_strategy_oracle import CASES, NAMES, check_against_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


@pytest.mark.parametrize("name", CASES)
def test_refine_matches_reference(name):
    from gsplat_hip import densify
    g = load_golden(name)
    T = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(DEV)  # noqa: E731
    params = {k: T(g[f"in_{k}"]) for k in NAMES}
    moments = {k: [T(g[f"in_m_{k}"]), T(g[f"in_v_{k}"])] for k in NAMES}
    cfg = densify.DefaultStrategyConfig(revised_opacity=bool(g["revised"]))
    r2d = T(g["radii2d"]) if "radii2d" in g else None
    p, m, counts = densify.refine(params, moments, T(g["grad2d"]), T(g["count"]), int(g["step"]),
                                  cfg, scene_scale=float(g["scene_scale"]), z=T(g["z"]),
                                  radii2d=r2d)
    if int(g["reset"]):
        densify.reset_opacity(p, m, cfg.prune_opa * 2.0)
    torch.cuda.synchronize()
    check_against_golden(g, {k: v.cpu().numpy() for k, v in p.items()},
                         {k: [t.cpu().numpy() for t in v] for k, v in m.items()}, counts)


def test_refine_empty_and_nothing_to_do():
    from gsplat_hip import densify
    cfg = densify.DefaultStrategyConfig()
    z = lambda n: torch.zeros(n, device=DEV)  # noqa: E731
    params = {"means": z((0, 3)), "scales": z((0, 3)), "quats": z((0, 4)), "opacities": z(0)}
    p, m, c = densify.refine(params, {}, z(0), z(0), 600, cfg)
    assert c == (0, 0, 0) and all(v.shape[0] == 0 for v in p.values())
    # low gradients, opaque, mid-sized: everything kept in order, moments copied
    N = 777
    params = {"means": torch.randn(N, 3, device=DEV), "scales": torch.full((N, 3), -3.0, device=DEV),
              "quats": torch.randn(N, 4, device=DEV), "opacities": torch.full((N,), 2.0, device=DEV),
              "shN": torch.randn(N, 15, 3, device=DEV)}
    moms = {k: [torch.rand_like(v), torch.rand_like(v)] for k, v in params.items()}
    p, m, c = densify.refine(params, moms, z(N), torch.ones(N, device=DEV), 700, cfg)
    assert c == (0, 0, 0)
    for k in params:
        assert torch.equal(p[k], params[k]) and torch.equal(m[k][0], moms[k][0])


def test_refine_large_matches_oracle():
    """100k Gaussians with degree-3 SH rows (the trainer's layout), noise
    drawn on the device: the HIP compaction equals the oracle's."""
    from gsplat_hip import densify
    from oracle import strategy_oracle as S
    gen = torch.Generator().manual_seed(5)
    N = 100_000
    params = {"means": torch.randn(N, 3, generator=gen),
              "scales": torch.rand(N, 3, generator=gen) * 5.7 - 6.9,
              "quats": torch.randn(N, 4, generator=gen),
              "opacities": torch.randn(N, generator=gen) * 3 - 2,
              "sh0": torch.randn(N, 1, 3, generator=gen), "shN": torch.randn(N, 15, 3, generator=gen)}
    moms = {k: [torch.rand(v.shape, generator=gen), torch.rand(v.shape, generator=gen)]
            for k, v in params.items()}
    count = torch.randint(0, 6, (N,), generator=gen).float()
    grad2d = torch.rand(N, generator=gen) * 6e-4 * count
    cfg = densify.DefaultStrategyConfig()
    dg = torch.Generator(device=DEV).manual_seed(11)
    dp = {k: v.to(DEV) for k, v in params.items()}
    dm = {k: [t.to(DEV) for t in v] for k, v in moms.items()}
    p, m, c = densify.refine(dp, dm, grad2d.to(DEV), count.to(DEV), 3500, cfg, generator=dg)
    n_split = c[1]
    z = torch.randn(2, n_split, 3, device=DEV, generator=torch.Generator(device=DEV).manual_seed(11))
    rp, rm, rc = S.refine({k: v.numpy() for k, v in params.items()},
                          {k: (a.numpy(), b.numpy()) for k, (a, b) in moms.items()},
                          grad2d.numpy(), count.numpy(), 3500, z.cpu().numpy())
    assert c == rc
    for k in params:
        got = p[k].cpu().numpy()
        if k in ("means", "scales"):
            np.testing.assert_allclose(got, rp[k], rtol=2e-6, atol=1e-6, err_msg=k)
        else:
            np.testing.assert_array_equal(got, rp[k], err_msg=k)
        np.testing.assert_array_equal(m[k][0].cpu().numpy(), rm[k][0], err_msg=k)
        np.testing.assert_array_equal(m[k][1].cpu().numpy(), rm[k][1], err_msg=k)
