"""GPU: the sync-free tile intersection and the training step replayed as a
HIP graph (gsplat_hip/graph_step.py).

* capacity-mode isect (gsplat_hip_isect_write_sorted_capped): the written
  isects are bit-identical to the synchronous path's, offsets and renders
  too; on overflow nothing is written, the counts say so and the sticky
  status flag is set;
* the device-side Adam factors (gsplat_hip_adam_step_dev,
  gsplat_hip_sh_colors_bwd_adam_dev) give the same bits as the host-scalar
  launches, and a set void flag updates nothing;
* the graph-replayed trainer tracks the eager trainer (the rasterizer's
  float atomics make two runs differ in the last bits), also when its isect
  capacity is too small at first: the overflowed steps are voided, the
  capacity grows, the step is re-captured and the void steps re-run."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def _scene(N=30000, W=640, H=480, seed=2):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * torch.tensor([1.6, 1.2, 0.6])
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.06 + 0.004
    opac = torch.rand(N, generator=g)
    sh = torch.randn(N, 16, 3, generator=g) * 0.3
    vm = torch.eye(4)[None]
    K = torch.tensor([[500.0, 0, W / 2], [0, 500.0, H / 2], [0, 0, 1]])[None]
    return [x.to(DEV) for x in (means, quats, scales, opac, sh, vm, K)], W, H


def _render(ins, W, H, **kw):
    import gsplat_hip
    leaves = [x.clone().requires_grad_(True) for x in ins[:5]]
    rc, ra, meta = gsplat_hip.rasterization(*leaves, ins[5], ins[6], W, H, sh_degree=3,
                                            packed=False, **kw)
    w = torch.rand(rc.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
    (rc * w).sum().backward()
    torch.cuda.synchronize()
    return rc.detach(), ra.detach(), meta, [x.grad for x in leaves]


def test_capped_isect_matches_synchronous():
    ins, W, H = _scene()
    rc0, ra0, m0, g0 = _render(ins, W, H)
    n = m0["flatten_ids"].numel()
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    rc1, ra1, m1, g1 = _render(ins, W, H, _isect_capacity=n + 12345, _isect_status=status)
    counts = m1["isect_counts"].tolist()
    assert counts[0] == n and counts[2] == 0 and counts[3] == n and int(status) == 0
    assert counts[1] == int((m0["tiles_per_gauss"] > 0).sum())
    assert m1["isect_ids"].numel() == n + 12345
    assert torch.equal(m1["isect_ids"][:n], m0["isect_ids"])
    assert torch.equal(m1["flatten_ids"][:n], m0["flatten_ids"])
    assert torch.equal(m1["isect_offsets"], m0["isect_offsets"])
    # the same per-tile lists through the same deterministic forward
    assert torch.equal(rc1, rc0) and torch.equal(ra1, ra0)
    for a, b in zip(g1, g0):  # the backward's float atomics: summation order only
        scale = float(b.abs().max())
        assert float((a - b).abs().max()) <= 5e-5 * scale + 1e-9
    # exactly full is not an overflow
    _, _, m2, _ = _render(ins, W, H, _isect_capacity=n, _isect_status=status)
    assert m2["isect_counts"].tolist()[2] == 0 and int(status) == 0
    assert torch.equal(m2["isect_ids"], m0["isect_ids"])


def test_capped_isect_flatten_only_2dgs():
    """The 2DGS training step's capped isect (ABI 33: `_colors_only`, no
    64-bit isect ids): the flatten ids and offsets written equal the
    synchronous emission's, isect_ids comes back None, and the render is the
    same (the colours-only render of the same per-tile lists)."""
    import gsplat_hip
    ins, W, H = _scene(N=20000)
    vm, K = ins[5], ins[6]
    out0 = gsplat_hip.rasterization_2dgs(*ins[:5], vm, K, W, H, sh_degree=3,
                                         render_mode="RGB+D", _colors_only=True)
    m0 = out0[-1]
    n = m0["flatten_ids"].numel()
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    out1 = gsplat_hip.rasterization_2dgs(*ins[:5], vm, K, W, H, sh_degree=3,
                                         render_mode="RGB+D", _colors_only=True,
                                         _isect_capacity=n + 777, _isect_status=status)
    m1 = out1[-1]
    counts = m1["isect_counts"].tolist()
    assert counts[0] == n and counts[2] == 0 and int(status) == 0
    from gsplat_hip import _lib
    if _lib.query("gsplat_hip_isect_ranked", 1, m0["tile_width"], m0["tile_height"]):
        assert m1["isect_ids"] is None
    assert torch.equal(m1["flatten_ids"][:n], m0["flatten_ids"])
    assert torch.equal(m1["isect_offsets"], m0["isect_offsets"])
    assert torch.equal(out1[0], out0[0]) and torch.equal(out1[1], out0[1])


def test_capped_isect_overflow_writes_nothing():
    ins, W, H = _scene(N=8000)
    _, _, m0, _ = _render(ins, W, H)
    n = m0["flatten_ids"].numel()
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    rc, ra, m1, grads = _render(ins, W, H, _isect_capacity=n - 1, _isect_status=status)
    written, _, over, total = m1["isect_counts"].tolist()
    assert (written, over, total) == (0, 1, n) and int(status) == 1
    assert int(m1["isect_offsets"].abs().sum()) == 0  # every tile empty
    assert float(ra.abs().max()) == 0.0 and torch.isfinite(rc).all()
    assert all(torch.isfinite(g).all() for g in grads)
    # sticky: a later render that fits leaves the flag set
    _render(ins, W, H, _isect_capacity=2 * n, _isect_status=status)
    assert int(status) == 1


def test_adam_device_factors_are_exact():
    """adam_factors + gsplat_hip_adam_step_dev == gsplat_hip_adam_step, bit
    for bit, over steps and a changing learning rate; a void step changes
    nothing."""
    from gsplat_hip.losses import adam_factors, adam_groups
    torch.manual_seed(3)
    shapes = [(4099, 3), (4099, 4), (4099,), (4099, 15, 3)]
    lrs = [1.6e-4, 1e-3, 5e-2, 1.25e-4]
    betas, eps = (0.9, 0.999), 1e-15
    base = [torch.randn(s, device=DEV) for s in shapes]
    res = []
    for dev_form in (False, True):
        ps = [b.clone() for b in base]
        ms = [torch.zeros_like(b) for b in base]
        vs = [torch.zeros_like(b) for b in base]
        hyper = torch.zeros(2 * len(shapes), device=DEV)
        void = torch.zeros(1, dtype=torch.int32, device=DEV)
        for step in range(1, 6):
            g = torch.Generator(device=DEV).manual_seed(step)
            grads = [torch.randn(s, device=DEV, generator=g) for s in shapes]
            lr_t = [lr * (0.99 ** step) for lr in lrs]
            flat = lambda ts: [t.view(-1) for t in ts]  # noqa: E731
            if dev_form:
                hyper.copy_(torch.tensor([x for f in adam_factors(lr_t, betas, step) for x in f]))
                adam_groups(flat(ps), flat(grads), flat(ms), flat(vs), lr_t, betas, eps, 0,
                            hyper=hyper, skip=void)
            else:
                adam_groups(flat(ps), flat(grads), flat(ms), flat(vs), lr_t, betas, eps, step)
        if dev_form:  # a void step
            before = [p.clone() for p in ps]
            void.fill_(1)
            adam_groups(flat(ps), flat(grads), flat(ms), flat(vs), lr_t, betas, eps, 0,
                        hyper=hyper, skip=void)
            assert all(torch.equal(a, b) for a, b in zip(before, ps))
        torch.cuda.synchronize()
        res.append(ps + ms + vs)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_sh_adam_device_factors_are_exact():
    from gsplat_hip import _wrapper
    from gsplat_hip.losses import FusedAdam, adam_factors
    g = torch.Generator(device=DEV).manual_seed(9)
    N = 2049
    means = torch.randn(N, 3, device=DEV, generator=g) * 2
    vm = torch.eye(4, device=DEV)[None]
    vm[0, 2, 3] = 6.0
    radii = (torch.rand(1, N, device=DEV, generator=g) > 0.4).int() * 3
    sh0 = torch.randn(N, 1, 3, device=DEV, generator=g) * 0.3
    shN = torch.randn(N, 15, 3, device=DEV, generator=g) * 0.1
    ws = [torch.rand(1, N, 3, device=DEV, generator=g) - 0.5 for _ in range(3)]
    res = []
    for dev_form in (False, True):
        p0, p1 = sh0.clone().requires_grad_(True), shN.clone().requires_grad_(True)
        opt = FusedAdam([p0, p1], [2.5e-3, 1.25e-4], eps=1e-15)
        hyper = torch.zeros(3, device=DEV)
        void = torch.zeros(1, dtype=torch.int32, device=DEV)
        for it in range(3):
            step = opt.step_count + 1
            if dev_form:
                (s0, ib), (sr, _) = adam_factors(opt.lrs, opt.betas, step)
                hyper.copy_(torch.tensor([s0, sr, ib]))
                fa = _wrapper.ShAdamInBackward(p0.data, p1.data, opt.exp_avg[0],
                                               opt.exp_avg_sq[0], opt.exp_avg[1],
                                               opt.exp_avg_sq[1], opt.lrs[0], opt.lrs[1],
                                               opt.betas, opt.eps, 1, hyper=hyper, skip=void)
            else:
                fa = _wrapper.ShAdamInBackward(p0.data, p1.data, opt.exp_avg[0],
                                               opt.exp_avg_sq[0], opt.exp_avg[1],
                                               opt.exp_avg_sq[1], opt.lrs[0], opt.lrs[1],
                                               opt.betas, opt.eps, step)
            colors = _wrapper.sh_colors(3, means, vm, (p0, p1), radii,
                                        fusion=_wrapper.StepFusion(sh_adam=fa))
            (colors * ws[it]).sum().backward()
            assert fa.applied
            opt.step_count += 1
        torch.cuda.synchronize()
        res.append((p0.detach().clone(), p1.detach().clone(), *opt.exp_avg, *opt.exp_avg_sq))
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def _trainer_scene(n_cams=3, W=320, H=240, stride=8):
    """The garden crop's every `stride`-th point at W x H.  stride 8: 13,974
    Gaussians, tiles of <= 554 isects; stride 1 (heavy tiles): 111,785
    Gaussians, ~280 k isects, 32-38 tiles above 2048 isects per camera --
    above the split threshold, so the trainer runs the split forward."""
    import os
    from gsplat_hip.train_step import camera_pool, load_garden_scene
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(root, "tests", "golden", "garden_scene.npz"), scene_grid=1)
    means, rgbs = means[::stride].contiguous(), rgbs[::stride].contiguous()
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=n_cams)
    return means, rgbs, vm, K, W, H


@pytest.mark.parametrize("capacity,stride", [(None, 8), (1000, 8), (None, 1), (20000, 1)])
def test_graph_trainer_tracks_eager(capacity, stride):
    """Six replayed steps against six eager ones, with the library's adaptive
    split forward on: the trainer picks the forward variant once, from its
    first render (Trainer.split_launch), so eager and captured renders run
    the same kernel.  stride 1: heavy tiles, the split forward runs (its
    chunks' products are exercised in both).  The rasterizer backward's float
    atomics still make two eager runs differ in the last bits and grad2d sums
    gradient norms that can cancel: its bar comes from the spread of two
    eager runs (measured here)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene(stride=stride)
    out = {}
    for run in ("eager", "eager2", "graph"):
        graph = run == "graph"
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=graph,
                     isect_capacity=capacity, max_steps=100)
        assert (tr._graph is not None) == graph
        losses = [tr.step(it) for it in range(6)]
        tr.sync()
        assert tr.graph_fallback is None, tr.graph_fallback
        assert tr.split_launch == (1 if stride == 1 else 0), (tr.split_launch, tr.max_tile_first)
        out[run] = ({k: p.detach().clone() for k, p in tr.params.items()},
                    [m.clone() for m in tr.opt.exp_avg], tr.opt.step_count,
                    tr.grad2d.clone(), tr.count.clone(), [float(x) for x in losses])
        if graph:
            g = tr._graph
            assert g.replays >= 6
            if capacity is not None:  # started too small: grown and re-captured
                assert g.recaptures >= 2 and g.capacity > g.max_isects > capacity
    a, a2, b = out["eager"], out["eager2"], out["graph"]
    assert a[2] == b[2] == 6
    for k in a[0]:
        torch.testing.assert_close(b[0][k], a[0][k], rtol=1e-3, atol=1e-5)
    for x, y in zip(a[1], b[1]):
        torch.testing.assert_close(y, x, rtol=1e-2, atol=1e-6)
    torch.testing.assert_close(b[4], a[4], rtol=0, atol=0)  # visibility counts: exact
    spread = float((a2[3] - a[3]).abs().max())
    err = float((b[3] - a[3]).abs().max())
    print(f"grad2d: graph-vs-eager {err:.3e}, eager run-to-run {spread:.3e}, "
          f"max {float(a[3].abs().max()):.3e}")
    assert err <= max(4.0 * spread, 1e-5 * float(a[3].abs().max())), (err, spread)
    # the returned per-step losses (the graph's loss ring slots): with a tiny
    # capacity too, where the voided steps' redo writes the returned slots
    torch.testing.assert_close(torch.tensor(b[5]), torch.tensor(a[5]), rtol=1e-4, atol=1e-6)
    assert len(set(b[5])) == 6, b[5]


@pytest.mark.parametrize("capacity", [None, 1000])
def test_graph_2dgs_trainer_tracks_eager(capacity):
    """The 2DGS (surfel) trainer's step captured and replayed (configs[4]):
    rasterization_2dgs with the sync-free isect and the surfel rasterizer
    reading the isect count on the device; with a tiny capacity the voided
    steps re-run.  Six replayed steps against six eager ones, grad2d at the
    run-to-run spread of two eager runs (float atomics of the backward)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene()
    out = {}
    for run in ("eager", "eager2", "graph"):
        graph = run == "graph"
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, model="2dgs", graph=graph,
                     isect_capacity=capacity, max_steps=100)
        assert (tr._graph is not None) == graph
        losses = [tr.step(it) for it in range(6)]
        tr.sync()
        assert tr.graph_fallback is None, tr.graph_fallback
        out[run] = ({k: p.detach().clone() for k, p in tr.params.items()},
                    [m.clone() for m in tr.opt.exp_avg], tr.opt.step_count,
                    tr.grad2d.clone(), tr.count.clone(), [float(x) for x in losses])
        if graph:
            g = tr._graph
            assert g.replays >= 6
            assert set(g.census) <= {"kernel", "empty"}, g.census
            if capacity is not None:
                assert g.recaptures >= 2 and g.capacity > g.max_isects > capacity
    a, a2, b = out["eager"], out["eager2"], out["graph"]
    assert a[2] == b[2] == 6
    torch.testing.assert_close(torch.tensor(b[5]), torch.tensor(a[5]), rtol=1e-4, atol=1e-6)
    assert len(set(b[5])) == 6, b[5]
    for k in a[0]:
        torch.testing.assert_close(b[0][k], a[0][k], rtol=1e-3, atol=1e-5)
    for x, y in zip(a[1], b[1]):
        torch.testing.assert_close(y, x, rtol=1e-2, atol=1e-6)
    torch.testing.assert_close(b[4], a[4], rtol=0, atol=0)
    # grad2d sums float-atomic gradients over six steps: single cancelling
    # elements may differ by more than two eager runs happen to (2.6e-6
    # against a spread of 2.3e-7 seen, with the voided steps' re-runs): the
    # bulk within 4x the eager spread, a few outliers within 1e-3 of the max
    spread = float((a2[3] - a[3]).abs().max())
    gmax = float(a[3].abs().max())
    err = (b[3] - a[3]).abs()
    bar = max(4.0 * spread, 1e-5 * gmax)
    print(f"grad2d: graph-vs-eager {float(err.max()):.3e}, eager run-to-run {spread:.3e}, "
          f"{int((err > bar).sum())} of {err.numel()} above {bar:.3e}")
    assert int((err > bar).sum()) <= max(2, err.numel() // 2000), (float(err.max()), spread)
    assert float(err.max()) <= 1e-3 * gmax, (float(err.max()), gmax)


def test_graph_trainer_refine_tracks_eager():
    """A DefaultStrategy schedule (refines at steps 3 and 6, opacity resets at
    0 and 7): the graph-replayed trainer re-captures after every refine (new
    parameter tensors) and its sequence of updates -- the refines' counts
    included -- follows the eager trainer's."""
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene()
    cfg = DefaultStrategyConfig(refine_start_iter=1, refine_every=3, reset_every=7)
    out = {}
    for graph in (False, True):
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=graph, max_steps=100,
                     strategy=cfg)
        assert (tr._graph is not None) == graph
        for it in range(9):
            tr.step(it)
        tr.sync()
        out[graph] = ({k: p.detach().clone() for k, p in tr.params.items()},
                      list(tr.refine_log), tr.opt.step_count, tr.grad2d.clone(),
                      tr.count.clone())
        if graph:
            g = tr._graph
            assert g.replays >= 9 and g.recaptures >= 3  # first capture + one per refine
    a, b = out[False], out[True]
    assert [r[0] for r in a[1]] == [3, 6] and a[1] == b[1], (a[1], b[1])
    assert a[2] == b[2] == 9
    for k in a[0]:
        torch.testing.assert_close(b[0][k], a[0][k], rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(b[4], a[4], rtol=0, atol=0)
    torch.testing.assert_close(b[3], a[3], rtol=1e-3, atol=1e-7)


def test_captured_step_holds_kernel_nodes_only():
    """Every capture is checked (graph_step.check_kernel_nodes_only): the
    replayed step holds kernel nodes, no memset / memcpy nodes (DESIGN
    §3.12); the returned loss is a copy that later replays do not touch."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene()
    tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=True, max_steps=100)
    l0 = tr.step(0)
    v0 = float(l0)
    tr.step(1)
    tr.sync()
    census = tr._graph.census
    assert set(census) <= {"kernel", "empty"} and census["kernel"] > 20, census
    assert float(l0) == v0


def test_loss_target_index_is_exact():
    """l1_ssim_loss(gt_index=...): the target picked on the device from a
    stack gives the loss and gradient of that target passed directly."""
    from gsplat_hip.losses import l1_ssim_loss
    g = torch.Generator(device=DEV).manual_seed(11)
    stack = torch.rand(4, 96, 128, 3, device=DEV, generator=g)
    img = torch.rand(1, 96, 128, 3, device=DEV, generator=g)
    for ci in (0, 3):
        a = img.clone().requires_grad_(True)
        b = img.clone().requires_grad_(True)
        la = l1_ssim_loss(a, stack[ci:ci + 1].contiguous())
        lb = l1_ssim_loss(b, stack, gt_index=torch.tensor([ci], device=DEV))
        la.backward()
        lb.backward()
        assert torch.equal(la.detach(), lb.detach()) and torch.equal(a.grad, b.grad)


def test_graph_recapture_failure_reruns_voided_steps(monkeypatch):
    """A recovery (isect overflow: grow, re-capture, redo) whose re-capture
    fails: the voided steps run eagerly, in order, before the current one,
    their losses land in the tensors already returned for them, and the
    trainer continues eagerly -- the same update sequence as an eager run
    (no step lost)."""
    from gsplat_hip import graph_step
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene()
    ref = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=False, max_steps=100)
    la = [float(ref.step(it)) for it in range(6)]
    ref.sync()
    orig = graph_step.GraphStep._capture_impl
    calls = []

    def second_fails(self, deg, stats=True):
        calls.append(1)
        if len(calls) >= 2:
            raise RuntimeError("injected re-capture failure")
        return orig(self, deg, stats)

    monkeypatch.setattr(graph_step.GraphStep, "_capture_impl", second_fails)
    tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=True, isect_capacity=1000,
                 max_steps=100)
    with pytest.warns(UserWarning, match="eagerly"):
        ret = [tr.step(it) for it in range(6)]
    tr.sync()
    assert tr._graph is None and "injected" in tr.graph_fallback
    assert tr.opt.step_count == 6 and len(calls) == 2
    lb = [float(x) for x in ret]
    for x, y in zip(la, lb):
        assert abs(x - y) <= 1e-4 * abs(x), (la, lb)
    for k in ref.params:
        torch.testing.assert_close(tr.params[k].detach(), ref.params[k].detach(), rtol=1e-3,
                                   atol=1e-5)
    torch.testing.assert_close(tr.count, ref.count, rtol=0, atol=0)


def test_graph_trainer_sh_adam_unfused_tracks_eager(monkeypatch):
    """GSPLAT_HIP_SH_ADAM_IN_BWD=0 with the geometry update in the projection
    backward: the launched groups (sh0, shN) take their device-side factors
    from the launch plan's tail (not the geometry's) -- replays equal eager
    steps."""
    from gsplat_hip.train_step import Trainer
    monkeypatch.setenv("GSPLAT_HIP_SH_ADAM_IN_BWD", "0")
    means, rgbs, vm, K, W, H = _trainer_scene()
    out = {}
    for graph in (False, True):
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=graph, max_steps=100)
        assert not tr.sh_adam_in_bwd and tr.geom_in_proj
        losses = [float(tr.step(it)) for it in range(5)]
        tr.sync()
        assert tr.graph_fallback is None, tr.graph_fallback
        assert (tr._graph is not None) == graph
        out[graph] = (losses, {k: p.detach().clone() for k, p in tr.params.items()})
    torch.testing.assert_close(torch.tensor(out[True][0]), torch.tensor(out[False][0]),
                               rtol=1e-4, atol=1e-6)
    for k in out[False][1]:
        torch.testing.assert_close(out[True][1][k], out[False][1][k], rtol=1e-3, atol=1e-5)
