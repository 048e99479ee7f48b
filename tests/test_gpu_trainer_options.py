"""GPU: simple_trainer options on the trainer.
* visible_adam (simple_trainer.py:263-266,782-797): SelectiveAdam -- the
  reference's Adam kernel, no bias correction, applied only to the rows of
  the Gaussians the step's camera sees, (radii > 0).any(0) -- through
  gsplat_hip_selective_adam, one launch per parameter group;
* packed (simple_trainer.py:123,501): the render's [nnz] pairs and the
  strategy statistics by index_add over gaussian_ids (default.py:240-254)
  train as the dense [C, N] path does;
* sparse_grad (simple_trainer.py:125,263-264,767-780): COO gradients over
  the pairs' Gaussians and torch.optim.SparseAdam;
* antialiased (simple_trainer.py:129,482): rasterize_mode "antialiased",
  eager and graph-replayed."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def test_trainer_visible_adam():
    from gsplat_hip._wrapper_aux import SelectiveAdam
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", visible_adam=True, graph=True)
    assert isinstance(tr.opt, SelectiveAdam) and tr._graph is None  # eager steps
    assert not tr.sh_adam_in_bwd and not tr.geom_fuse and not tr.geom_in_proj
    with torch.no_grad():
        _, _, meta = tr.render(tr.camera_index(0), tr.sh_degree_at(0))
    vis = meta["radii"] > 0
    if vis.dim() > 2:
        vis = vis.all(-1)
    vis = vis.any(0)
    assert 0 < int(vis.sum()) < vis.numel()  # some seen, some not
    p0 = {k: p.detach().clone() for k, p in tr.params.items()}
    loss = tr.step(0)
    assert math.isfinite(float(loss))
    b1, b2 = tr.adam_kw["betas"]
    for (k, p), lr in zip(tr.params.items(), tr.lrs):
        d = (p.detach() - p0[k]).reshape(p.shape[0], -1)
        st = tr.opt.state[p]
        m = st["exp_avg"].reshape(p.shape[0], -1)
        # rows no camera saw: untouched, moments still zero
        assert torch.equal(d[~vis], torch.zeros_like(d[~vis])), k
        assert torch.equal(m[~vis], torch.zeros_like(m[~vis])), k
        # seen rows with a gradient: the first step without bias correction
        # moves by lr (1 - b1) / sqrt(1 - b2) against the gradient's sign
        sel = vis[:, None] & (m.abs() > 1e-10)
        if int(sel.sum()) == 0:
            continue
        ratio = d[sel].abs() / lr
        expect = (1 - b1) / math.sqrt(1 - b2)
        assert abs(float(ratio.median()) - expect) < 1e-3 * expect, (k, float(ratio.median()))
        assert bool((torch.sign(d[sel]) == -torch.sign(m[sel])).all()), k
    for it in range(1, 4):
        assert math.isfinite(float(tr.step(it)))


def test_trainer_packed_tracks_dense():
    """Packed against dense training, with DefaultStrategy statistics
    accumulating (no refine yet).  After the first step (same parameters in):
    the loss, grad2d (to 1e-4 of its largest entry: the backward's float
    atomics summed in another order) and the visibility counts (exact).  After four:
    the parameters, where Adam's normalised step can turn a last-bit
    difference of a near-zero gradient into up to 2 lr per step, so each
    entry within 2 lr per step and all but a few within 1e-6."""
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    cfg = DefaultStrategyConfig(refine_start_iter=100)
    out = {}
    for run in ("dense", "dense2", "packed"):
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", strategy=cfg, max_steps=100,
                     packed=run == "packed", graph=True)
        assert (tr._graph is None) == (run == "packed")
        loss0 = float(tr.step(0))
        tr.sync()
        first = (loss0, tr.grad2d.clone(), tr.count.clone())
        for it in range(1, 4):
            tr.step(it)
        tr.sync()
        out[run] = (first, {k: p.detach().clone() for k, p in tr.params.items()}, list(tr.lrs))
    a, a2, b = out["dense"], out["dense2"], out["packed"]
    assert abs(b[0][0] - a[0][0]) <= 1e-5 * abs(a[0][0]), (a[0][0], b[0][0])
    torch.testing.assert_close(b[0][2], a[0][2], rtol=0, atol=0)  # visibility counts
    spread = float((a2[0][1] - a[0][1]).abs().max())
    err = float((b[0][1] - a[0][1]).abs().max())
    # (packed rows put the backward's per-Gaussian atomics in another order
    # than the dense rows do: sums of cancelling tile contributions move by
    # ~1e-5 of the largest entry, where two dense runs agree to 1e-8)
    assert err <= max(4.0 * spread, 1e-4 * float(a[0][1].abs().max())), (err, spread)
    for (k, x), lr in zip(a[1].items(), a[2]):
        d = (b[1][k] - x).abs()
        assert float(d.max()) <= 2 * lr * 4 * 1.001, (k, float(d.max()), lr)
        assert float((d > 1e-6).float().mean()) < 0.01, (k, float((d > 1e-6).float().mean()))


def test_trainer_sparse_grad():
    """sparse_grad with packed: every parameter's gradient is COO over the
    step's gaussian_ids, SparseAdam leaves the other rows and their moments
    alone, and a refine (DefaultStrategy) carries the SparseAdam state."""
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    # (no strategy for the first step's checks: DefaultStrategy resets every
    # opacity at step 0, as the reference's, default.py:195)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", packed=True, sparse_grad=True,
                 max_steps=100)
    assert isinstance(tr.opt, torch.optim.SparseAdam) and tr._graph is None
    with torch.no_grad():
        _, _, meta = tr.render(tr.camera_index(0), tr.sh_degree_at(0))
    seen = torch.zeros(means.shape[0], dtype=torch.bool, device="cuda")
    seen[meta["gaussian_ids"]] = True
    assert 0 < int(seen.sum()) < seen.numel()
    p0 = {k: p.detach().clone() for k, p in tr.params.items()}
    assert math.isfinite(float(tr.step(0)))
    for k, p in tr.params.items():
        d = (p.detach() - p0[k]).reshape(p.shape[0], -1)
        assert torch.equal(d[~seen], torch.zeros_like(d[~seen])), k  # rows no pair touched
        assert float(d[seen].abs().max()) > 0, k
        m = tr.opt.state[p]["exp_avg"].reshape(p.shape[0], -1)
        assert float(m[~seen].abs().max()) == 0.0, k
    cfg = DefaultStrategyConfig(refine_start_iter=1, refine_every=2, reset_every=100)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", packed=True, sparse_grad=True,
                 strategy=cfg, max_steps=100)
    for it in range(0, 5):  # refines at 2 and 4
        assert math.isfinite(float(tr.step(it)))
        n = tr.params["means"].shape[0]
        for k, (m, v) in tr.moments().items():
            assert m.shape == tr.params[k].shape and v.shape[0] == n, k
    assert [r[0] for r in tr.refine_log] == [2, 4], tr.refine_log


def test_trainer_antialiased_graph_tracks_eager():
    """rasterize_mode "antialiased" (the projection's compensations scale
    the opacities): the trainer's render equals rasterization() called with
    that mode, and four replayed steps track four eager ones (the geometry
    Adam stays out of the projection backward, which fuses only classic)."""
    from gsplat_hip import rasterization
    from gsplat_hip.train_step import Trainer
    from test_gpu_trainer import _small_scene
    means, rgbs, vm, K, W, H = _small_scene()
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", antialiased=True)
    with torch.no_grad():
        c, _, meta = tr.render(0, 3)
        p = tr.params
        ref, _, _ = rasterization(p["means"], p["quats"], torch.exp(p["scales"]),
                                  torch.sigmoid(p["opacities"]),
                                  torch.cat([p["sh0"], p["shN"]], 1), tr.viewmats[:1],
                                  tr.Ks[:1], W, H, sh_degree=3, packed=False,
                                  rasterize_mode="antialiased")
    assert meta["opacities"].shape == (1, means.shape[0])
    torch.testing.assert_close(c, ref, rtol=1e-4, atol=1e-5)
    out = {}
    for run in ("eager", "eager2", "graph"):
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", antialiased=True,
                     graph=run == "graph", max_steps=100)
        assert (tr._graph is not None) == (run == "graph")
        losses = [tr.step(it) for it in range(4)]
        tr.sync()
        assert tr.graph_fallback is None, tr.graph_fallback
        out[run] = ({k: q.detach().clone() for k, q in tr.params.items()},
                    [float(x) for x in losses])
    a, a2, b = out["eager"], out["eager2"], out["graph"]
    for k in a[0]:
        spread = float((a2[0][k] - a[0][k]).abs().max())
        err = float((b[0][k] - a[0][k]).abs().max())
        assert err <= max(4.0 * spread, 1e-5 * float(a[0][k].abs().max()) + 1e-6), (k, err, spread)
    torch.testing.assert_close(torch.tensor(b[1]), torch.tensor(a[1]), rtol=1e-4, atol=1e-6)
