"""MCMCStrategy on the CPU: the oracle (oracle/mcmc_oracle.py) against the
reference's own step_post_backward (tests/golden/mcmc_*.npz, made by
tests/golden/make_golden_mcmc.py with the reference's draws recorded), the
config / schedule of gsplat_hip.mcmc, and the sampler above torch's 2^24
category limit.  The HIP path is tests/test_gpu_mcmc.py."""

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mcmc_oracle as M

NAMES = ("means", "scales", "quats", "opacities", "sh0", "shN")
CASES = ("mcmc_refine", "mcmc_cap", "mcmc_alive", "mcmc_noise")


def golden_inputs(g):
    params = {k: g[f"in_{k}"] for k in NAMES}
    moments = {k: [g[f"in_m_{k}"], g[f"in_v_{k}"]] for k in NAMES}
    return params, moments


@pytest.mark.parametrize("case", CASES)
def test_oracle_vs_reference_golden(case):
    g = load_golden(case)
    params, moments = golden_inputs(g)
    p, m = M.step(params, moments, int(g["step"]), float(g["lr"]), g["z"], g["reloc_idx"],
                  g["add_idx"], cap_max=int(g["cap_max"]), noise_lr=float(g["noise_lr"]),
                  min_opacity=float(g["min_opacity"]))
    for k in NAMES:
        assert p[k].shape == g[f"out_{k}"].shape, k
        # scales / opacities of relocated rows pass through Eq. 9 in float64
        # here and float32 in the golden's restated kernel: 1e-4 relative
        np.testing.assert_allclose(p[k], g[f"out_{k}"], rtol=1e-4, atol=1e-5, err_msg=k)
        np.testing.assert_array_equal(m[k][0], g[f"out_m_{k}"], err_msg=k)
        np.testing.assert_array_equal(m[k][1], g[f"out_v_{k}"], err_msg=k)


def test_golden_cases_cover_the_branches():
    r, c, a, n = (load_golden(k) for k in CASES)
    assert r["refine"] and r["n_dead"] > 0 and len(r["add_idx"]) == 50
    assert c["refine"] and len(c["add_idx"]) == 20  # min(cap_max 820, 1.05 * 800) - 800
    assert a["refine"] and a["n_dead"] == 0 and len(a["reloc_idx"]) == 0
    assert not n["refine"] and n["out_means"].shape == n["in_means"].shape
    assert not np.array_equal(n["out_means"], n["in_means"])  # the noise moved something


def test_config_matches_reference_defaults():
    from gsplat_hip.mcmc import MCMCStrategyConfig
    c = MCMCStrategyConfig()
    # gsplat/strategy/mcmc.py:49-55
    assert (c.cap_max, c.noise_lr, c.refine_start_iter, c.refine_stop_iter, c.refine_every,
            c.min_opacity, c.verbose) == (1_000_000, 5e5, 500, 25_000, 100, 0.005, False)
    # mcmc.py:122-126: strictly inside (start, stop), on multiples of refine_every
    steps = [s for s in range(0, 26_000) if c.is_refine_step(s)]
    assert steps[0] == 600 and steps[-1] == 24_900 and len(steps) == 244


def test_binoms_and_n_to_add():
    from gsplat_hip import mcmc
    b = mcmc.binoms()
    assert b.shape == (51, 51) and b[50, 25] == float(__import__("math").comb(50, 25))
    assert torch.equal(b, torch.from_numpy(M.binoms()))
    assert mcmc.n_to_add(1000, 1_000_000) == 50
    assert mcmc.n_to_add(800, 820) == 20
    assert mcmc.n_to_add(900, 820) == 0  # above the cap: nothing (never negative)


def test_multinomial_above_torch_limit():
    """ops.py:29-44 switches to numpy above 2^24 categories; here inverse CDF
    on the tensor's device -- draws land only where the weight is non-zero,
    in proportion."""
    from gsplat_hip.mcmc import multinomial_sample
    n = 2 ** 24 + 7
    w = torch.zeros(n)
    hot = torch.tensor([0, 5, 2 ** 24 + 6])
    w[hot] = torch.tensor([1.0, 2.0, 1.0])
    gen = torch.Generator().manual_seed(0)
    s = multinomial_sample(w, 40_000, gen)
    assert s.dtype == torch.int64 and s.shape == (40_000,)
    assert torch.isin(s, hot).all()
    frac = torch.stack([(s == h).float().mean() for h in hot])
    assert torch.allclose(frac, torch.tensor([0.25, 0.5, 0.25]), atol=0.02)
    small = multinomial_sample(w[:100], 10, gen)  # torch.multinomial below the limit
    assert torch.isin(small, torch.tensor([0, 5])).all()
