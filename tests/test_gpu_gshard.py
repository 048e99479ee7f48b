"""GPU: Gaussian-sharded multi-GPU training (rasterization(distributed=True),
Trainer(gaussian_shard=True)) at world size 2 -- two processes sharing the
one GPU of the box, talking over gloo (the exchange stages GPU tensors
through host memory there; on a node RCCL moves them over xGMI).

* each rank renders its own camera with both ranks' Gaussians: the images
  equal a one-process render of the whole scene, and each rank's local
  gradients equal the whole-scene gradients of the two cameras' summed loss
  at its Gaussians [rank::2] (float atomics: last bits);
* one trainer step per rank equals one whole-scene step that renders both
  cameras, sums their losses and runs Adam with the batch-2 hyperparameters
  (simple_trainer.py:261-277) -- the reference's multi-GPU training step.
"""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(N=24000, W=320, H=240, seed=5):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * torch.tensor([1.4, 1.0, 0.6])
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.05 + 0.005
    opac = torch.rand(N, generator=g)
    sh0 = torch.randn(N, 1, 3, generator=g) * 0.3
    shN = torch.randn(N, 15, 3, generator=g) * 0.05
    vm = torch.eye(4).repeat(2, 1, 1)
    vm[1, 0, 3] = 0.3
    K = torch.tensor([[300.0, 0, W / 2], [0, 300.0, H / 2], [0, 0, 1]]).repeat(2, 1, 1)
    w = torch.rand(2, H, W, 3, generator=g) - 0.5
    return (means, quats, scales, opac, sh0, shN), vm, K, w, W, H


def _render_rank(rank, world, port, out_dir):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        import gsplat_hip
        ins, vm, K, w, W, H = _scene()
        N = ins[0].shape[0]
        local = [t[rank::world].contiguous().to(DEV).requires_grad_(True) for t in ins]
        n_world = [len(range(r, N, world)) for r in range(world)]
        rc, ra, meta = gsplat_hip.rasterization(
            local[0], local[1], local[2], local[3], (local[4], local[5]),
            vm[rank:rank + 1].to(DEV), K[rank:rank + 1].to(DEV), W, H, sh_degree=3,
            packed=False, distributed=True,
            _world_cameras=(vm.to(DEV), K.to(DEV)), _world_counts=n_world)
        (rc * w[rank:rank + 1].to(DEV)).sum().backward()
        torch.cuda.synchronize()
        torch.save({"rc": rc.detach().cpu(), "ra": ra.detach().cpu(),
                    "grads": [t.grad.cpu() for t in local],
                    "n_cameras": meta["n_cameras"], "radii": meta["radii"].cpu()},
                   os.path.join(out_dir, f"render{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_gshard_render_matches_whole_scene(tmp_path):
    import torch.multiprocessing as mp
    import gsplat_hip
    from test_gpu_parity import close_most
    mp.spawn(_render_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    ins, vm, K, w, W, H = _scene()
    full = [t.to(DEV).requires_grad_(True) for t in ins]
    rc, ra, meta = gsplat_hip.rasterization(
        full[0], full[1], full[2], full[3], (full[4], full[5]), vm.to(DEV), K.to(DEV), W, H,
        sh_degree=3, packed=False)
    (rc * w.to(DEV)).sum().backward()
    for r in range(2):
        got = torch.load(os.path.join(tmp_path, f"render{r}.pt"), weights_only=True)
        assert got["n_cameras"] == 1
        assert torch.equal(got["radii"], meta["radii"][:, r::2].cpu())  # [C_world, N_local]
        # the same Gaussians per tile in the same depth order: ties aside, the same image
        close_most(got["rc"][0], rc[r], 1e-5, 1e-5, f"colors rank {r}")
        close_most(got["ra"][0], ra[r], 1e-5, 1e-5, f"alphas rank {r}")
        for name, a, t in zip(("means", "quats", "scales", "opacities", "sh0", "shN"),
                              got["grads"], full):
            b = t.grad[r::2].cpu()
            scale = max(1e-12, float(b.abs().max()))
            close_most(a, b, 1e-3, 1e-4 * scale, f"{name} grad rank {r}", rows=a.dim() > 1,
                       out_bound=0.05 * scale)


def _trainer_rank(rank, world, port, out_dir):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from gsplat_hip.train_step import Trainer
        means, rgbs, vm, K, W, H = _trainer_scene()
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, world_size=world, rank=rank,
                     gaussian_shard=True)
        assert tr.gshard and not tr.sharded and tr.sh_adam_in_bwd and tr.geom_fuse
        tr.step(0)
        tr.sync()
        torch.save({"params": {k: p.detach().cpu() for k, p in tr.params.items()},
                    "count": tr.count.cpu(), "grad2d": tr.grad2d.cpu(),
                    "n_world": tr._n_world},
                   os.path.join(out_dir, f"trainer{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _trainer_scene(W=320, H=240, trim=0):
    from gsplat_hip.train_step import camera_pool, load_garden_scene
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=1)
    means, rgbs = means[::8].contiguous(), rgbs[::8].contiguous()
    if trim:  # 13974 points split evenly three ways; 13973 do not
        means, rgbs = means[:-trim].contiguous(), rgbs[:-trim].contiguous()
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=4)
    return means, rgbs, vm, K, W, H


def test_gshard_trainer_step_matches_whole_scene_step(tmp_path):
    import math
    import torch.multiprocessing as mp
    from gsplat_hip.losses import FusedAdam, l1_ssim_loss
    from gsplat_hip.rendering import rasterization
    from gsplat_hip.strategy import update_state_
    from gsplat_hip.train_step import Trainer
    from test_gpu_parity import close_most
    mp.spawn(_trainer_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    means, rgbs, vm, K, W, H = _trainer_scene()
    # the whole scene, initialised as the shards were (same generator draws)
    ref = Trainer(means, rgbs, vm, K, W, H, device=DEV, world_size=1, fused=True)
    params = {k: torch.nn.Parameter(p.detach().clone()) for k, p in ref.params.items()}
    N = params["means"].shape[0]
    BS = 2
    lrs = [Trainer.LRS[k] * math.sqrt(BS) for k in params]
    opt = FusedAdam(list(params.values()), lrs, eps=1e-15 / math.sqrt(BS),
                    betas=(1 - BS * (1 - 0.9), 1 - BS * (1 - 0.999)))
    grad2d = torch.zeros(N, device=DEV)
    count = torch.zeros(N, device=DEV)
    loss = 0.0
    metas = []
    for ci in (0, 1):  # step 0: rank r renders camera (0 * 2 + r) % n = r
        scales, opac = torch.exp(params["scales"]), torch.sigmoid(params["opacities"])
        colors, _, meta = rasterization(
            params["means"], params["quats"], scales, opac, (params["sh0"], params["shN"]),
            vm[ci:ci + 1].to(DEV), K[ci:ci + 1].to(DEV), W, H, sh_degree=3, packed=False,
            near_plane=0.01, far_plane=1e10, radius_clip=0.0)
        meta["means2d"].retain_grad()
        metas.append(meta)
        loss = loss + l1_ssim_loss(colors, ref.targets[ci:ci + 1], 0.2)
    loss.backward()
    for meta in metas:
        update_state_(grad2d, count, meta["means2d"].grad, meta["radii"], W, H, 1)
    opt.step()
    for r in range(2):
        got = torch.load(os.path.join(tmp_path, f"trainer{r}.pt"), weights_only=True)
        assert got["n_world"] == [len(range(0, N, 2)), len(range(1, N, 2))]
        assert torch.equal(got["count"], count[r::2].cpu())
        close_most(got["grad2d"], grad2d[r::2].cpu(), 1e-4, 1e-6, f"grad2d rank {r}")
        for k, p in params.items():
            b = p.detach()[r::2].cpu()
            a = got["params"][k]
            assert a.shape == b.shape, (k, a.shape, b.shape)
            # Adam's first step moves each entry by about +-lr: a gradient
            # within rounding of zero may take either sign (a few entries)
            close_most(a, b, 1e-5, 1e-6, f"{k} rank {r}", max_frac=2e-3,
                       out_bound=2.5 * lrs[list(params).index(k)])


def _trainer_rank_refine(rank, world, port, out_dir):
    """World-`world` Gaussian-sharded trainer, uneven shards, a refine at step
    1 (each shard refined alone, then the shard sizes all-gathered), then a
    step with the new shard sizes."""
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from gsplat_hip import densify, train_step
        from gsplat_hip.densify import DefaultStrategyConfig
        from gsplat_hip.train_step import Trainer
        means, rgbs, vm, K, W, H = _trainer_scene(trim=1)
        # one refine, at step 1 (steps below refine_stop_iter = 2)
        cfg = DefaultStrategyConfig(refine_start_iter=0, refine_every=1, refine_stop_iter=2,
                                    reset_every=10 ** 6, grow_grad2d=2e-5)
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, world_size=world, rank=rank,
                     gaussian_shard=True, strategy=cfg)
        n0 = tr.params["means"].shape[0]
        saved = {}
        orig = densify.refine

        def spy(params, moments, grad2d, count, step, *a, **kw):
            saved.update(params={k: v.detach().cpu().clone() for k, v in params.items()},
                         grad2d=grad2d.cpu().clone(), count=count.cpu().clone(), step=step)
            return orig(params, moments, grad2d, count, step, *a, **kw)
        train_step.densify.refine = spy
        try:
            tr.step(0)
            tr.step(1)  # refine
        finally:
            train_step.densify.refine = orig
        loss = float(tr.step(2))
        tr.sync()
        torch.save({"n0": n0, "n1": tr.params["means"].shape[0], "n_world": tr._n_world,
                    "log": tr.refine_log, "pre": saved, "loss": loss},
                   os.path.join(out_dir, f"refine{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_gshard_trainer_refine_world3(tmp_path):
    """Three ranks on the one GPU (gloo), shards [r::3] of uneven sizes: the
    per-shard refines make the whole scene's decisions (the refine on the
    re-interleaved shards' statistics gives the same duplicate / split /
    prune counts), every rank all-gathers the same new shard sizes, and the
    next step runs with them."""
    import torch.multiprocessing as mp
    from gsplat_hip import densify
    from gsplat_hip.densify import DefaultStrategyConfig
    world = 3
    mp.spawn(_trainer_rank_refine, args=(world, _port(), str(tmp_path)), nprocs=world,
             join=True)
    got = [torch.load(os.path.join(tmp_path, f"refine{r}.pt"), weights_only=True)
           for r in range(world)]
    N = sum(g["n0"] for g in got)
    assert N % world != 0 and len({g["n0"] for g in got}) == 2  # uneven shards
    sizes = [g["n1"] for g in got]
    for g in got:
        assert g["n_world"] == sizes
        assert [e[0] for e in g["log"]] == [1] and np.isfinite(g["loss"])
    # the whole scene's refine decisions from the shards' inputs, re-interleaved
    def whole(key, sub=None):
        parts = [g["pre"][key] if sub is None else g["pre"][key][sub] for g in got]
        out = torch.empty((N,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype)
        for r, p in enumerate(parts):
            out[r::world] = p
        return out.to(DEV)
    params = {k: whole("params", k).contiguous() for k in got[0]["pre"]["params"]}
    moments = {k: [torch.zeros_like(v), torch.zeros_like(v)] for k, v in params.items()}
    cfg = DefaultStrategyConfig(refine_start_iter=0, refine_every=1, refine_stop_iter=2,
                                reset_every=10 ** 6, grow_grad2d=2e-5)
    _, _, counts = densify.refine(params, moments, whole("grad2d").contiguous(),
                                  whole("count").contiguous(), 1, cfg, 1.0,
                                  generator=torch.Generator(device=DEV).manual_seed(0))
    per_rank = [g["log"][0][1:4] for g in got]
    assert tuple(counts) == tuple(sum(c[i] for c in per_rank) for i in range(3)), \
        (counts, per_rank)
    assert sum(counts) > 0


def _sh_case(C=5, N=3001, seed=3):
    g = torch.Generator(device=DEV).manual_seed(seed)
    means = torch.randn(N, 3, device=DEV, generator=g) * 2
    vm = torch.eye(4, device=DEV).repeat(C, 1, 1)
    vm[:, 2, 3] = 6.0 + torch.arange(C, device=DEV)
    vm[:, 0, 3] = torch.linspace(-1, 1, C, device=DEV)
    radii = (torch.rand(C, N, device=DEV, generator=g) > 0.5).int() * 2
    sh0 = torch.randn(N, 1, 3, device=DEV, generator=g) * 0.3
    shN = torch.randn(N, 15, 3, device=DEV, generator=g) * 0.1
    vcol = torch.rand(C, N, 3, device=DEV, generator=g) - 0.5
    return means, vm, radii, sh0, shN, vcol


def test_sh_backward_summed_over_cameras():
    """gsplat_hip_sh_colors_bwd_sum (C cameras sharing the coefficient rows,
    summed in registers) against the per-camera rows of gsplat_hip_sh_colors_bwd
    summed by torch."""
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    for C in (1, 2, 5):
        means, vm, radii, sh0, shN, vcol = _sh_case(C)
        N = means.shape[0]
        per0 = torch.empty(C, N, 1, 3, device=DEV)
        perr = torch.empty(C, N, 15, 3, device=DEV)
        perd = torch.empty(C, N, 3, device=DEV)
        _lib.call("gsplat_hip_sh_colors_bwd", 3, C, N, N, 16, _ptr(means), _ptr(vm), _ptr(sh0),
                  _ptr(shN), _ptr(radii), _ptr(vcol), _ptr(per0), _ptr(perr), _ptr(perd),
                  _stream())
        s0 = torch.empty(N, 1, 3, device=DEV)
        sr = torch.empty(N, 15, 3, device=DEV)
        sd = torch.empty(N, 3, device=DEV)
        _lib.call("gsplat_hip_sh_colors_bwd_sum", 3, C, N, _ptr(means), _ptr(vm), _ptr(sh0),
                  _ptr(shN), _ptr(radii), _ptr(vcol), _ptr(s0), _ptr(sr), _ptr(sd), _stream())
        torch.cuda.synchronize()
        # the same arithmetic per camera; the compiler may contract the basis
        # polynomials differently in the two kernels (last bits)
        for a, b in ((s0, per0.sum(0)), (sr, perr.sum(0)), (sd, perd.sum(0))):
            torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-7)


def test_sh_adam_in_backward_over_cameras_is_exact():
    """The fused SH Adam with C cameras == the summed gradient + FusedAdam,
    bit for bit (the same in-register sum, the shared element update)."""
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    from gsplat_hip.losses import adam_groups
    C = 4
    means, vm, radii, sh0, shN, vcol = _sh_case(C, N=2048)
    N = means.shape[0]
    out = []
    for fused in (False, True):
        p0, pr = sh0.clone(), shN.clone()
        m0, v0 = torch.zeros_like(p0), torch.zeros_like(p0)
        mr, vr = torch.zeros_like(pr), torch.zeros_like(pr)
        vd = torch.empty(N, 3, device=DEV)
        for step in (1, 2, 3):
            if fused:
                _lib.call("gsplat_hip_sh_colors_bwd_adam", 3, C, N, _ptr(means), _ptr(vm),
                          _ptr(p0), _ptr(pr), _ptr(radii), _ptr(vcol), _ptr(vd), _ptr(m0),
                          _ptr(v0), _ptr(mr), _ptr(vr), 2.5e-3, 1.25e-4, 0.9, 0.999, 1e-15,
                          step, _stream())
            else:
                g0 = torch.empty_like(p0)
                gr = torch.empty_like(pr)
                _lib.call("gsplat_hip_sh_colors_bwd_sum", 3, C, N, _ptr(means), _ptr(vm),
                          _ptr(p0), _ptr(pr), _ptr(radii), _ptr(vcol), _ptr(g0), _ptr(gr),
                          _ptr(vd), _stream())
                adam_groups([p0.view(-1), pr.view(-1)], [g0.view(-1), gr.view(-1)],
                            [m0.view(-1), mr.view(-1)], [v0.view(-1), vr.view(-1)],
                            [2.5e-3, 1.25e-4], (0.9, 0.999), 1e-15, step)
        torch.cuda.synchronize()
        out.append((p0, pr, m0, v0, mr, vr, vd))
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_emulated_rank0_render_matches_whole_scene():
    """bench.py --gshard-emulate: one process renders rank 0's camera of a
    world-2 job with rank 1's rows recorded from rank 1's own render -- the
    image of the whole scene, as the real two-rank render gives; the
    backward's emulated exchange runs and yields finite gradients."""
    import gsplat_hip
    from gsplat_hip import distributed as gdist
    from test_gpu_parity import close_most
    ins, vm, K, w, W, H = _scene()
    N = ins[0].shape[0]
    n_world = [len(range(r, N, 2)) for r in range(2)]

    def render(rank):
        local = [t[rank::2].contiguous().to(DEV).requires_grad_(True) for t in ins]
        out = gsplat_hip.rasterization(
            local[0], local[1], local[2], local[3], (local[4], local[5]),
            vm[rank:rank + 1].to(DEV), K[rank:rank + 1].to(DEV), W, H, sh_degree=3,
            packed=False, distributed=True, _world_cameras=(vm.to(DEV), K.to(DEV)),
            _world_counts=n_world)
        return out, local

    prev = gdist.EMULATION
    gdist.EMULATION = gdist.Emulation(2)
    try:
        gdist.EMULATION.record(1, lambda: render(1))
        (rc, ra, meta), local = render(0)
        (rc * w[0:1].to(DEV)).sum().backward()
        torch.cuda.synchronize()
    finally:
        gdist.EMULATION = prev
    full = [t.to(DEV) for t in ins]
    rf, af, _ = gsplat_hip.rasterization(full[0], full[1], full[2], full[3], (full[4], full[5]),
                                         vm[:1].to(DEV), K[:1].to(DEV), W, H, sh_degree=3,
                                         packed=False)
    close_most(rc[0].detach(), rf[0], 1e-5, 1e-5, "colors")
    close_most(ra[0].detach(), af[0], 1e-5, 1e-5, "alphas")
    assert all(t.grad is not None and torch.isfinite(t.grad).all() for t in local)


def test_graph_gshard_emulated_step_tracks_eager():
    """The Gaussian-sharded step replayed as a HIP graph (the pair exchanges
    inside it: the one-GPU emulation's device copies; graph_step.graphable):
    rank 0 of an emulated 3-rank job, four steps, the world's cameras from
    the step block, against the same steps issued eagerly."""
    from gsplat_hip import distributed as gdist
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _trainer_scene(trim=1)
    world = 3
    saved = gdist.EMULATION
    try:
        gdist.EMULATION = gdist.Emulation(world)
        for j in range(1, world):
            peer = Trainer(means, rgbs, vm, K, W, H, device=DEV, world_size=world, rank=j,
                           gaussian_shard=True, graph=False)
            gdist.EMULATION.record(j, lambda: peer.render(peer.camera_index(0),
                                                          peer.sh_degree_at(0)))
            del peer
        out = {}
        for graph in (False, True):
            tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, world_size=world, rank=0,
                         gaussian_shard=True, graph=graph, max_steps=100)
            assert (tr._graph is not None) == graph
            for it in range(4):
                tr.step(it)
            tr.sync()
            out[graph] = ({k: p.detach().clone() for k, p in tr.params.items()},
                          tr.count.clone(), tr.grad2d.clone())
            if graph:
                assert tr._graph.replays >= 4 and set(tr._graph.census) <= {"kernel", "empty"}
    finally:
        gdist.EMULATION = saved
    a, b = out[False], out[True]
    for k in a[0]:
        torch.testing.assert_close(b[0][k], a[0][k], rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(b[1], a[1], rtol=0, atol=0)
    torch.testing.assert_close(b[2], a[2], rtol=1e-3, atol=1e-7)
