"""GPU: MCMCStrategy on the HIP backend (gsplat_hip.mcmc; relocation and the
fused position noise in csrc/aux_ops.hip) against the reference's own
step_post_backward (tests/golden/mcmc_*.npz, its draws recorded and fed
back), the noise kernel against the reference's torch formula at 1M
Gaussians, and the Trainer's MCMC schedule.

Bars: the optimizer moments and every copied row exact; relocated
opacities / scales (Eq. 9 in float32 here, float64 in the oracle the golden
used) and the noised means within 1e-4 relative."""

import math

import numpy as np
import pytest
import torch

from conftest import load_golden
from test_mcmc import CASES, NAMES

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def T(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(DEV)


@pytest.mark.parametrize("case", CASES)
def test_step_matches_reference(case):
    from gsplat_hip import mcmc
    g = load_golden(case)
    cfg = mcmc.MCMCStrategyConfig(cap_max=int(g["cap_max"]))
    params = {k: T(g[f"in_{k}"]) for k in NAMES}
    moms = {k: [T(g[f"in_m_{k}"]), T(g[f"in_v_{k}"])] for k in NAMES}
    b = mcmc.binoms(DEV)
    step = int(g["step"])
    assert cfg.is_refine_step(step) == bool(g["refine"])
    if cfg.is_refine_step(step):
        dead = torch.sigmoid(params["opacities"]) <= cfg.min_opacity
        n = mcmc.relocate(params, moms, dead, b, cfg.min_opacity, sampled=T(g["reloc_idx"]))
        assert n == int(g["n_dead"])
        n_add = mcmc.n_to_add(params["means"].shape[0], cfg.cap_max)
        assert n_add == len(g["add_idx"])
        if n_add:
            params, moms = mcmc.sample_add(params, moms, n_add, b, cfg.min_opacity,
                                           sampled=T(g["add_idx"]))
    mcmc.inject_noise(params, float(g["lr"]) * cfg.noise_lr, z=T(g["z"]))
    torch.cuda.synchronize()
    for k in NAMES:
        out = params[k].cpu().numpy()
        assert out.shape == g[f"out_{k}"].shape, k
        np.testing.assert_allclose(out, g[f"out_{k}"], rtol=1e-4, atol=1e-5, err_msg=k)
        np.testing.assert_array_equal(moms[k][0].cpu().numpy(), g[f"out_m_{k}"], err_msg=k)
        np.testing.assert_array_equal(moms[k][1].cpu().numpy(), g[f"out_v_{k}"], err_msg=k)
    # rows the refine did not touch are bit-identical (copies, no arithmetic)
    if not int(g["refine"]):
        for k in NAMES[1:]:
            np.testing.assert_array_equal(params[k].cpu().numpy(), g[f"out_{k}"])


def _noise_reference(means, quats, log_scales, logits, z, scaler):
    """ops.py:350-369 in torch fp32 (covariance as _torch_impl.py:49-53)."""
    q = quats / quats.norm(dim=-1, keepdim=True)
    w, x, y, zq = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + zq * zq), 2 * (x * y - w * zq), 2 * (x * zq + w * y),
                     2 * (x * y + w * zq), 1 - 2 * (x * x + zq * zq), 2 * (y * zq - w * x),
                     2 * (x * zq - w * y), 2 * (y * zq + w * x), 1 - 2 * (x * x + y * y)],
                    -1).reshape(-1, 3, 3)
    M = R * torch.exp(log_scales)[:, None, :]
    cov = torch.bmm(M, M.transpose(-1, -2))
    o = torch.sigmoid(logits)
    f = 1 / (1 + torch.exp(-100 * ((1 - o) - 0.995)))
    return means + torch.einsum("bij,bj->bi", cov, z * f[:, None] * scaler)


def test_noise_kernel_1m_vs_torch():
    from gsplat_hip import mcmc
    gen = torch.Generator(device=DEV).manual_seed(11)
    N = 1_000_000
    p = {"means": torch.randn(N, 3, device=DEV, generator=gen),
         "quats": torch.randn(N, 4, device=DEV, generator=gen),
         "scales": torch.rand(N, 3, device=DEV, generator=gen) * 4 - 6,
         "opacities": torch.randn(N, device=DEV, generator=gen) * 3 - 3}
    z = torch.randn(N, 3, device=DEV, generator=gen)
    ref = _noise_reference(p["means"], p["quats"], p["scales"], p["opacities"], z, 80.0)
    before = p["means"].clone()
    mcmc.inject_noise(p, 80.0, z=z)
    d_ref, d = ref - before, p["means"] - before
    assert float(d.abs().max()) > 1e-4  # the low-opacity rows really move
    # the displacement to 1e-4 of its largest entry (fp32 op order differs)
    assert float((d - d_ref).abs().max()) <= 1e-4 * float(d_ref.abs().max()) + 1e-7
    # the generator path draws z itself; scaler 0: nothing moves
    after = p["means"].clone()
    mcmc.inject_noise(p, 0.0, generator=gen)
    assert torch.equal(p["means"], after)


def test_inject_noise_to_position_dropin():
    """The reference signature (ops.py:343-369) and draw: torch.randn_like
    from the global generator, so a seeded run moves the means as the
    reference's torch formula does with the same seed."""
    from gsplat_hip import mcmc
    gen = torch.Generator(device=DEV).manual_seed(3)
    N = 50_000
    params = {"means": torch.nn.Parameter(torch.randn(N, 3, device=DEV, generator=gen)),
              "quats": torch.nn.Parameter(torch.randn(N, 4, device=DEV, generator=gen)),
              "scales": torch.nn.Parameter(torch.rand(N, 3, device=DEV, generator=gen) * 4 - 6),
              "opacities": torch.nn.Parameter(torch.randn(N, device=DEV, generator=gen) * 3 - 3)}
    before = params["means"].detach().clone()
    torch.manual_seed(77)
    z = torch.randn_like(params["means"])
    ref = _noise_reference(before, params["quats"].detach(), params["scales"].detach(),
                           params["opacities"].detach(), z, 80.0)
    torch.manual_seed(77)
    mcmc.inject_noise_to_position(params, optimizers={}, state={}, scaler=80.0)
    d_ref, d = ref - before, params["means"].detach() - before
    assert float((d - d_ref).abs().max()) <= 1e-4 * float(d_ref.abs().max()) + 1e-7


def test_noise_kernel_empty_and_misaligned_quats():
    from gsplat_hip import mcmc
    e = {"means": torch.zeros(0, 3, device=DEV), "quats": torch.zeros(0, 4, device=DEV),
         "scales": torch.zeros(0, 3, device=DEV), "opacities": torch.zeros(0, device=DEV)}
    mcmc.inject_noise(e, 1.0)
    N = 1000
    buf = torch.randn(4 * N + 1, device=DEV)
    q = buf[1:].view(N, 4)  # 4-B offset: re-aligned by the wrapper
    p = {"means": torch.zeros(N, 3, device=DEV), "quats": q,
         "scales": torch.full((N, 3), -3.0, device=DEV), "opacities": torch.full((N,), -8.0, device=DEV)}
    z = torch.randn(N, 3, device=DEV)
    ref = _noise_reference(p["means"], q, p["scales"], p["opacities"], z, 5.0)
    mcmc.inject_noise(p, 5.0, z=z)
    torch.testing.assert_close(p["means"], ref, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("graph", [False, True])
def test_trainer_mcmc_schedule(graph):
    """simple_trainer.py's mcmc preset (opacity / scale regularisers 0.01) on
    the HIP path, compressed in time: relocate + add on steps 2, 4, 6, capped;
    each refine leaves no dead Gaussian, rebuilds parameters and Adam state
    consistently, and the noise runs every step (graph=True: inside the
    replays between the eager refines)."""
    from gsplat_hip.mcmc import MCMCStrategyConfig
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    n0 = means.shape[0]
    cap = n0 + n0 // 20 + n0 // 40  # the second add is capped, the third adds nothing
    cfg = MCMCStrategyConfig(refine_start_iter=1, refine_every=2, cap_max=cap)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", strategy=cfg, max_steps=100,
                 opacity_reg=0.01, scale_reg=0.01, graph=graph)
    assert (tr._graph is not None) == graph
    # a few certainly dead Gaussians to relocate at the first refine
    tr.params["opacities"].data[:7] = -9.0
    losses = []
    for it in range(7):
        m0 = tr.params["means"].detach().clone()
        losses.append(float(tr.step(it)))
        n = tr.params["means"].shape[0]
        for k, p in tr.params.items():
            assert p.shape[0] == n, k
        for k, (m, v) in tr.moments().items():
            assert m.shape == tr.params[k].shape and v.shape == tr.params[k].shape, k
        if it in (2, 4, 6):
            o = torch.sigmoid(tr.params["opacities"].detach())
            assert int((o < cfg.min_opacity * 0.999).sum()) == 0, it
        elif n == m0.shape[0]:
            assert not torch.equal(tr.params["means"].detach(), m0)  # Adam + noise moved them
    assert [r[0] for r in tr.refine_log] == [2, 4, 6], tr.refine_log
    assert tr.refine_log[0][1] >= 7  # the forced dead ones at least
    n1 = n0 + max(0, min(cap, int(1.05 * n0)) - n0)
    n2 = n1 + max(0, min(cap, int(1.05 * n1)) - n1)
    assert [r[3] for r in tr.refine_log] == [n1, n2, n2], (tr.refine_log, n0, cap)
    assert [r[2] for r in tr.refine_log] == [n1 - n0, n2 - n1, 0]
    assert all(math.isfinite(x) for x in losses), losses
    assert "MCMCStrategy" in tr.densify_desc()
    tr.sync()
    if graph:
        assert tr.graph_fallback is None, tr.graph_fallback
        assert tr._graph.replays >= 7 and tr._graph.recaptures >= 3  # + one after each refine


def _unit_scene(N, logit=-12.0):
    """Sigma = I (identity rotation, unit scales) and opacity ~ 0: the
    displacement is z * op_sigmoid(1) * scaler."""
    p = {"means": torch.zeros(N, 3, device=DEV),
         "quats": torch.tensor([1.0, 0, 0, 0], device=DEV).repeat(N, 1),
         "scales": torch.zeros(N, 3, device=DEV), "opacities": torch.full((N,), logit, device=DEV)}
    o = torch.sigmoid(torch.tensor(logit))
    f = float(1 / (1 + torch.exp(-100 * ((1 - o) - 0.995))))
    return p, f


def test_noise_draw_in_kernel():
    """The trainer's draw (Philox-4x32-10 keyed by seed, counter (n, step),
    Box-Muller): standard normal per component, components and steps
    uncorrelated, a pure function of (seed, step, n); device step / scale /
    void flag as the captured step passes them."""
    from gsplat_hip import mcmc
    N = 1 << 20
    p, f = _unit_scene(N)
    mcmc.inject_noise(p, 1.0 / f, seed=1234, step=7)
    z = p["means"].clone()
    assert bool(torch.isfinite(z).all())
    m, sd = z.mean(0), z.std(0)
    assert float(m.abs().max()) < 5e-3 and float((sd - 1).abs().max()) < 5e-3, (m, sd)
    c = torch.corrcoef(z.T)
    assert float((c - torch.eye(3, device=DEV)).abs().max()) < 5e-3, c
    within = (z.abs() < 1).float().mean(0)
    assert float((within - 0.6827).abs().max()) < 3e-3, within
    assert float((z.abs() > 4).float().mean()) < 1e-4  # tails of a normal, no outliers
    # the same (seed, step): the same numbers; another step / seed: independent
    p2, _ = _unit_scene(N)
    mcmc.inject_noise(p2, 1.0 / f, seed=1234, step=7)
    assert torch.equal(p2["means"], z)
    for kw in (dict(seed=1234, step=8), dict(seed=1235, step=7)):
        p3, _ = _unit_scene(N)
        mcmc.inject_noise(p3, 1.0 / f, **kw)
        r = torch.corrcoef(torch.stack([p3["means"].reshape(-1), z.reshape(-1)]))[0, 1]
        assert abs(float(r)) < 5e-3, (kw, r)
    # device inputs: step and scale from memory, a zero scale or a void flag
    # moves nothing
    p4, _ = _unit_scene(N)
    sd_ = torch.tensor([7], dtype=torch.int64, device=DEV)
    sc = torch.tensor([1.0 / f], dtype=torch.float32, device=DEV)
    void = torch.zeros(1, dtype=torch.int32, device=DEV)
    mcmc.inject_noise(p4, 0.0, seed=1234, step=0, step_dev=sd_, scaler_dev=sc, skip=void)
    assert torch.equal(p4["means"], z)
    void.fill_(1)
    mcmc.inject_noise(p4, 0.0, seed=1234, step_dev=sd_, scaler_dev=sc, skip=void)
    void.zero_()
    sc.zero_()
    mcmc.inject_noise(p4, 0.0, seed=1234, step_dev=sd_, scaler_dev=sc, skip=void)
    assert torch.equal(p4["means"], z)


@pytest.mark.parametrize("capacity", [None, 1000])
def test_graph_mcmc_trainer_tracks_eager(capacity):
    """MCMC training as graph replays (the noise inside, step and scale from
    the step's input block) against eager steps: refines on steps 3 and 6
    (eager, re-captured after), the same Gaussian counts and parameters at
    the eager run-to-run spread; with a tiny isect capacity the voided steps
    re-run and draw the same noise."""
    from gsplat_hip.mcmc import MCMCStrategyConfig
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    cfg = MCMCStrategyConfig(refine_start_iter=2, refine_every=3)
    out = {}
    for run in ("eager", "eager2", "graph"):
        graph = run == "graph"
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, strategy=cfg, max_steps=100,
                     graph=graph, isect_capacity=capacity)
        assert (tr._graph is not None) == graph
        tr.params["opacities"].data[:5] = -9.0  # certainly dead at the first refine
        # (a returned loss of a voided step is rewritten by its re-run: read
        # them after the sync)
        losses = [tr.step(it) for it in range(8)]
        tr.sync()
        losses = [float(x) for x in losses]
        assert tr.graph_fallback is None, tr.graph_fallback
        out[run] = ({k: p.detach().clone() for k, p in tr.params.items()},
                    [r[1:] for r in tr.refine_log], losses)
        if graph:
            assert tr._graph.replays >= 8
    a, a2, b = out["eager"], out["eager2"], out["graph"]
    assert b[1] == a[1] == a2[1], (a[1], b[1])  # (relocated, added, N) per refine
    for k in a[0]:
        spread = float((a2[0][k] - a[0][k]).abs().max())
        err = float((b[0][k] - a[0][k]).abs().max())
        assert err <= max(4.0 * spread, 1e-5 * float(a[0][k].abs().max()) + 1e-6), (k, err, spread)
    torch.testing.assert_close(torch.tensor(b[2]), torch.tensor(a[2]), rtol=1e-4, atol=1e-6)
