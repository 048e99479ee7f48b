"""Per-camera data parallelism on CPU with gloo, world_size 2 (no GPU).

Covers the multi-GPU step's host logic with the same code bench.py runs over
RCCL: disjoint camera assignment per rank, the SUM all-reduce of every
Gaussian gradient group (Trainer.allreduce_grads), and the MAX-over-ranks
step time (bench.max_over_ranks)."""

import os
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from gsplat_hip.train_step import Trainer
        import bench

        # every group, incl. a missing gradient (None is skipped, as in training)
        shapes = {"means": (5, 3), "scales": (5, 3), "quats": (5, 4), "opacities": (5,),
                  "sh0": (5, 1, 3), "shN": (5, 15, 3)}
        params = {}
        for i, (k, shp) in enumerate(shapes.items()):
            p = torch.nn.Parameter(torch.zeros(shp))
            if k != "opacities":
                p.grad = torch.full(shp, float(rank + 1) * (i + 1))
            params[k] = p
        Trainer.allreduce_grads(SimpleNamespace(params=params))
        sums = {k: (None if p.grad is None else p.grad.unique().tolist())
                for k, p in params.items()}

        me = SimpleNamespace(world_size=WORLD, rank=rank, viewmats=torch.zeros(8, 4, 4))
        cams = [Trainer.camera_index(me, it) for it in range(4)]
        slow = bench.max_over_ranks(0.5 + rank, WORLD, "cpu")
        q.put((rank, sums, cams, slow))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the test
        q.put((rank, repr(e), None, None))


def test_dp_allreduce_cameras_and_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = dict()
    for _ in range(WORLD):
        rank, sums, cams, slow = q.get(timeout=120)
        out[rank] = (sums, cams, slow)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(WORLD):
        sums, cams, slow = out[rank]
        assert isinstance(sums, dict), sums
        for i, k in enumerate(["means", "scales", "quats", "opacities", "sh0", "shN"]):
            if k == "opacities":
                assert sums[k] is None
            else:  # (1 + 2) * (i + 1) on every rank
                assert sums[k] == [3.0 * (i + 1)], (k, sums[k])
        assert slow == 1.5  # the slower rank's time
    # per step, the ranks render different cameras; over steps all are used
    for it in range(4):
        assert out[0][1][it] != out[1][1][it]
    assert sorted(out[0][1] + out[1][1]) == list(range(8))


# ------------------------------------------------ Gaussian-sharded exchange --
def _comm_worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from gsplat_hip import distributed as gd
        out = {"ag": gd.all_gather_int32(WORLD, rank + 5, device="cpu"),
               "a2a": gd.all_to_all_int32(WORLD, [rank * 10, rank * 10 + 1], device="cpu")}
        # uneven splits: rank r sends r+1 rows to rank 0 and 2 rows to rank 1
        n0, n1 = rank + 1, 2
        a = (torch.arange(n0 + n1, dtype=torch.float32) + 100 * rank)[:, None].repeat(1, 3)
        a.requires_grad_(True)
        b = torch.full((n0 + n1,), float(rank))
        got = gd.all_to_all_int32(WORLD, [n0, n1], device="cpu")
        ra, rb = gd.all_to_all_tensor_list(WORLD, [a, b], [n0, n1], output_splits=got)
        (ra * torch.arange(1, ra.shape[0] + 1, dtype=torch.float32)[:, None]).sum().backward()
        out.update(got=got, ra=ra.detach()[:, 0].tolist(), rb=rb.tolist(), ga=a.grad[:, 0].tolist())
        g = gd.all_gather_tensor_list(WORLD, [torch.full((2, 4), float(rank))])
        out["gather"] = g[0][:, 0].tolist()
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the test
        q.put((rank, repr(e)))


def test_sharded_exchange_helpers_gloo():
    """gsplat_hip.distributed (the reference's gsplat/distributed.py surface)
    on two gloo ranks: integer gathers/exchanges, the differentiable
    many-to-many exchange with uneven splits (forward and backward)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(WORLD):
        assert isinstance(res[r], dict), res[r]
        assert res[r]["ag"] == [5, 6]
        assert res[r]["a2a"] == [r, 10 + r]
        assert res[r]["gather"] == [0.0, 0.0, 1.0, 1.0]
    # rank 0 receives rank 0's first row and rank 1's first two rows
    assert res[0]["got"] == [1, 2] and res[1]["got"] == [2, 2]
    assert res[0]["ra"] == [0.0, 100.0, 101.0] and res[0]["rb"] == [0.0, 1.0, 1.0]
    assert res[1]["ra"] == [1.0, 2.0, 102.0, 103.0]
    # d/da of sum(ra * row_index): the weights travel back to the senders
    # (row 0 lands at rank 0 position 0: weight 1; rows 1, 2 at rank 1 positions 0, 1)
    assert res[0]["ga"] == [1.0, 1.0, 2.0]
    assert res[1]["ga"] == [2.0, 3.0, 3.0, 4.0]


def test_reshape_view_blocks():
    """[sum_i C*N_i] blocks by source rank -> [C, sum_i N_i] (rendering.py:260-267)."""
    from gsplat_hip.rendering import _reshape_view
    C, N_world = 2, [2, 3]
    # rank 0 block: cameras 0,1 x its 2 Gaussians; rank 1: x its 3 Gaussians
    blk0 = torch.tensor([[0, 1], [10, 11]])
    blk1 = torch.tensor([[2, 3, 4], [12, 13, 14]])
    world = torch.cat([blk0.flatten(), blk1.flatten()])
    out = _reshape_view(C, world, N_world)
    assert out.tolist() == [[0, 1, 2, 3, 4], [10, 11, 12, 13, 14]]


def _sharded_worker(rank, world, port, q, defer=False, groups=None):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gsplat_hip.distributed import ShardedAdam, _adam_torch
        g = torch.Generator().manual_seed(0)  # identical replicas on every rank
        # row counts: divisible, with remainder rows, and fewer rows than ranks*4
        shapes = [(37, 15, 3), (37, 3), (37,), (40, 4), (5, 3)]
        init = [torch.randn(s, generator=g) for s in shapes]
        lrs = [1e-2, 2e-3, 5e-2, 1e-3, 3e-3]
        kw = dict(betas=(0.8, 0.99), eps=1e-8)
        ps = [torch.nn.Parameter(t.clone()) for t in init]
        ref = [t.clone() for t in init]
        opt = ShardedAdam(ps, lrs, update=_adam_torch, groups=groups, **kw)
        m = [torch.zeros_like(t).view(-1) for t in init]
        v = [torch.zeros_like(t).view(-1) for t in init]
        for step in range(1, 4):
            gr = torch.Generator().manual_seed(100 * step + rank)  # per-rank gradients
            grads = [torch.randn(s, generator=gr) for s in shapes]
            for p, gg in zip(ps, grads):
                p.grad = gg.clone()
            opt.step(defer_gather=defer)
            if defer:  # the trainer waits before the next use of the rows
                opt.wait()
            opt.zero_grad()
            # reference: all-reduce SUM of the gradients, full Adam on every rank
            summed = [gg.clone() for gg in grads]
            for t in summed:
                dist.all_reduce(t)
            _adam_torch([t.view(-1) for t in ref], [t.view(-1) for t in summed], m, v, lrs,
                        kw["betas"], kw["eps"], step)
        err = max(float((p.detach() - r).abs().max()) for p, r in zip(ps, ref))
        same = [p.detach().clone() for p in ps]
        q.put((rank, err, [t.tolist() for t in same]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e), None))


def _sharded_xform_worker(rank, world, port, q):
    """ShardedAdam with the trainer's DP configuration: two groups on two
    process groups, the second reduced early (reduce_early, as from the SH
    gradient hook), and gradient transforms (mode 1 summed before the
    reduction, modes 2 / 3 applied to the reduced shard)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gsplat_hip.distributed import ShardedAdam, _adam_torch
        g = torch.Generator().manual_seed(0)
        shapes = [(41, 3), (41, 3), (41, 4), (41,), (41, 1, 3), (41, 15, 3)]
        init = [torch.randn(s, generator=g) for s in shapes]
        lrs = [1.6e-4, 5e-3, 1e-3, 5e-2, 2.5e-3, 1.25e-4]
        kw = dict(betas=(0.9, 0.999), eps=1e-15)
        ps = [torch.nn.Parameter(t.clone()) for t in init]
        ref = [t.clone() for t in init]
        pg2 = dist.new_group(list(range(world)))
        opt = ShardedAdam(ps, lrs, update=_adam_torch, groups=[[0, 1, 2, 3], [4, 5]],
                          group_pgs=[None, pg2], **kw)
        m = [torch.zeros_like(t).view(-1) for t in init]
        v = [torch.zeros_like(t).view(-1) for t in init]
        for step in range(1, 4):
            gr = torch.Generator().manual_seed(100 * step + rank)
            grads = [torch.randn(s, generator=gr) for s in shapes]
            v_dirs = torch.randn(shapes[0], generator=gr)  # second means term
            s_act = torch.exp(ps[1].detach())             # replicated activations
            o_act = torch.sigmoid(ps[3].detach())
            for i in (0, 2, 4, 5):
                ps[i].grad = grads[i].clone()
            xf = {0: (ps[0].grad, v_dirs, 1), 1: (grads[1], s_act, 2), 3: (grads[3], o_act, 3)}
            opt.reduce_early(1)  # the SH group, before the rest
            opt.step(defer_gather=True, xform=xf)
            opt.wait()
            opt.zero_grad()
            # reference: all-reduce the per-rank gradients of the parameters
            # (VJPs on every rank's own gradient), full Adam
            loc = [grads[0] + v_dirs, grads[1] * s_act, grads[2], grads[3] * (1 - o_act) * o_act,
                   grads[4], grads[5]]
            for t in loc:
                dist.all_reduce(t)
            _adam_torch([t.view(-1) for t in ref], [t.view(-1) for t in loc], m, v, lrs,
                        kw["betas"], kw["eps"], step)
        err = max(float((p.detach() - r).abs().max() / (r.abs().max() + 1e-12))
                  for p, r in zip(ps, ref))
        q.put((rank, err, [p.detach().tolist() for p in ps]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None))


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_adam_dp_fusions_gloo(world):
    """The DP step's fusions: each group's collectives on its own process
    group, the SH group reduced early, the activation VJPs applied to the
    reduced shard (sum of VJPs == VJP of the sum up to rounding: 1e-5
    relative), replicas identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_xform_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, err, vals = q.get(timeout=180)
        out[rank] = (err, vals)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        err, vals = out[rank]
        assert not isinstance(err, str), err
        assert err < 1e-5, (rank, err)
        assert vals == out[0][1], "replicas diverged"


@pytest.mark.parametrize("world,defer,groups", [(2, False, None), (3, False, None),
                                               (2, True, None), (2, True, [[3, 1], [0, 2, 4]]),
                                               (3, False, [[2], [4, 0], [1, 3]]),
                                               (8, True, [[3, 1], [0, 2, 4]])])
def test_sharded_adam_matches_allreduce_adam_gloo(world, defer, groups):
    """ShardedAdam (reduce-scatter -> Adam on own rows -> all-gather) equals
    all-reduce + full Adam on every rank, and the replicas stay identical --
    also pipelined per parameter group (the trainer's geometry / SH split)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, defer, groups))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, err, vals = q.get(timeout=120)
        out[rank] = (err, vals)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        err, vals = out[rank]
        assert not isinstance(err, str), err
        assert err < 1e-5, (rank, err)
        assert vals == out[0][1], "replicas diverged"


# ------------------------------------------- densification under DP (gloo) --
def _oracle_refine(params, moments, grad2d, count, step, cfg, scene_scale=1.0, generator=None,
                   z=None, radii2d=None):
    """gsplat_hip.densify.refine's contract computed by the CPU oracle (the
    HIP kernels need a GPU): split noise drawn from `generator` exactly as the
    HIP path draws it (randn(2, n_split, 3) after the plan)."""
    import numpy as np
    from oracle import strategy_oracle as S
    grads = grad2d / count.clamp_min(1)
    high = grads > cfg.grow_grad2d
    split = high & (torch.exp(params["scales"]).max(-1).values > cfg.grow_scale3d * scene_scale)
    if radii2d is not None:
        split = split | (radii2d > cfg.grow_scale2d)
    n_split = int(split.sum())
    if z is None:
        z = torch.randn(2, n_split, 3, generator=generator)
    p, m, counts = S.refine({k: v.numpy() for k, v in params.items()},
                            {k: (a.numpy(), b.numpy()) for k, (a, b) in moments.items()},
                            grad2d.numpy(), count.numpy(), step, z.numpy(), scene_scale,
                            revised_opacity=cfg.revised_opacity,
                            radii2d=None if radii2d is None else radii2d.numpy())
    return ({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in p.items()},
            {k: [torch.from_numpy(np.ascontiguousarray(t)) for t in v] for k, v in m.items()},
            counts)


def _trainer_skeleton(rank, world, sharded, scale2d=False):
    """A Trainer with CPU parameters (no rendering): what refine touches."""
    from gsplat_hip import train_step
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.distributed import ShardedAdam, _adam_torch
    from gsplat_hip.losses import FusedAdam
    g = torch.Generator().manual_seed(0)  # identical replicas
    N = 203
    init = {"means": torch.randn(N, 3, generator=g),
            "scales": torch.rand(N, 3, generator=g) * 5.7 - 6.9,
            "quats": torch.randn(N, 4, generator=g),
            "opacities": torch.randn(N, generator=g) * 3 - 2,
            "sh0": torch.randn(N, 1, 3, generator=g), "shN": torch.randn(N, 15, 3, generator=g)}
    tr = train_step.Trainer.__new__(train_step.Trainer)
    tr.params = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
    tr.world_size, tr.rank, tr.device = world, rank, "cpu"
    tr.sharded, tr.fused = sharded, True
    tr.strategy = DefaultStrategyConfig(refine_scale2d_stop_iter=4000 if scale2d else 0)
    tr.scene_scale = 1.0
    tr.lrs = [1e-3] * 6
    tr.adam_kw = dict(betas=(0.9, 0.999), eps=1e-15)
    tr.rng = torch.Generator().manual_seed(42)
    tr.refine_log, tr.last_meta = [], None
    if sharded:
        tr.opt = ShardedAdam(list(tr.params.values()), tr.lrs, update=_adam_torch, **tr.adam_kw)
    else:
        tr.opt = FusedAdam.__new__(FusedAdam)
        tr.opt.params = list(tr.params.values())
        tr.opt.lrs, tr.opt.step_count = tr.lrs, 0
        tr.opt.exp_avg = [torch.zeros_like(p) for p in tr.opt.params]
        tr.opt.exp_avg_sq = [torch.zeros_like(p) for p in tr.opt.params]
    # populate the moments with two identical-on-every-rank Adam steps
    for step in range(2):
        gr = torch.Generator().manual_seed(7 + step)
        grads = [torch.randn(p.shape, generator=gr) * 1e-2 for p in tr.params.values()]
        if sharded:
            for p, gg in zip(tr.params.values(), grads):
                # the ranks' gradients sum to gg exactly (any world size)
                p.grad = gg if rank == 0 else torch.zeros_like(gg)
            tr.opt.step()
            tr.opt.zero_grad()
        else:
            tr.opt.step_count += 1
            _adam_torch([p.data.view(-1) for p in tr.opt.params], [x.view(-1) for x in grads],
                        [m.view(-1) for m in tr.opt.exp_avg],
                        [v.view(-1) for v in tr.opt.exp_avg_sq], tr.lrs,
                        tr.adam_kw["betas"], tr.adam_kw["eps"], tr.opt.step_count)
    # per-rank statistics (each rank saw its own cameras)
    gs = torch.Generator().manual_seed(100 + rank)
    tr.count = torch.randint(0, 4, (N,), generator=gs).float()
    tr.grad2d = torch.rand(N, generator=gs) * 4e-4 * tr.count
    # state["radii"] of this rank's cameras (MAX-reduced before the refine)
    tr.radii2d = torch.rand(N, generator=gs) ** 3 * 0.25 if scale2d else None
    return tr


def _refine_worker(rank, world, port, q, scale2d):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from gsplat_hip import train_step
        train_step.densify.refine = _oracle_refine
        tr = _trainer_skeleton(rank, world, sharded=True, scale2d=scale2d)
        tr.refine(3100)
        moms = tr.moments()  # all-gathered from the new shards
        # numpy, not tensors: a tensor in the queue lives in the worker's
        # shared memory, gone when the worker exits
        out = {"params": {k: v.detach().numpy().copy() for k, v in tr.params.items()},
               "m": {k: [t.numpy().copy() for t in v] for k, v in moms.items()},
               "log": tr.refine_log, "grad2d": float(tr.grad2d.abs().sum())}
        q.put((rank, out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world,scale2d", [(2, False), (2, True), (8, True)])
def test_refine_under_dp_keeps_replicas_identical_gloo(world, scale2d):
    """Trainer.refine on gloo ranks with different per-rank statistics: the
    statistics are summed (the screen radii MAX-reduced) before the decision,
    the split noise comes from the shared-seed generator, the sharded Adam
    moments are gathered, pushed through the compaction and re-sharded --
    every replica ends bit-identical and equal to a single-process refine on
    the combined statistics.  World 8 (configs[3]): 203 Gaussians give 24-row
    shards and 11 remainder rows (rows split in multiples of 4 * 8)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_refine_worker, args=(r, world, port, q, scale2d))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    for r in range(world):
        assert isinstance(res[r], dict), res[r]
    a = res[0]
    assert a["log"][0][0] == 3100
    for r in range(1, world):
        b = res[r]
        assert a["log"] == b["log"]
        for k in a["params"]:
            assert np.array_equal(a["params"][k], b["params"][k]), k
            assert np.array_equal(a["m"][k][0], b["m"][k][0])
            assert np.array_equal(a["m"][k][1], b["m"][k][1])
    assert a["grad2d"] == 0.0  # statistics restart after a refine

    # single process, unsharded, on the summed statistics: the same result
    import numpy as np  # noqa: F811
    from gsplat_hip import train_step
    saved = train_step.densify.refine
    train_step.densify.refine = _oracle_refine
    try:
        trs = [_trainer_skeleton(r, world, sharded=False, scale2d=scale2d)
               for r in range(world)]
        ref = trs[0]
        ref.world_size = 1
        # summed in rank order, as the ring reduction of the tests' gloo
        # group does for these small integers / exact sums
        ref.grad2d = sum((t.grad2d for t in trs[1:]), trs[0].grad2d.clone())
        ref.count = sum((t.count for t in trs[1:]), trs[0].count.clone())
        if scale2d:
            ref.radii2d = torch.stack([t.radii2d for t in trs]).amax(0)
        ref.refine(3100)
    finally:
        train_step.densify.refine = saved
    assert ref.refine_log == a["log"]
    for k, p in ref.params.items():
        np.testing.assert_array_equal(p.detach().numpy(), a["params"][k], err_msg=k)
        mm = ref.moments()[k]
        np.testing.assert_allclose(mm[0].numpy(), a["m"][k][0], rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(mm[1].numpy(), a["m"][k][1], rtol=1e-6, atol=1e-12)


PAIR_SHARDS = {2: [3, 2], 3: [4, 3, 3], 8: [3, 2, 3, 1, 2, 2, 3, 2]}  # uneven shards


def _pairs_worker(rank, port, q, world=WORLD):
    WORLD = world  # noqa: N806 (the module constant's role, per test)
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from gsplat_hip import distributed as gd
        from gsplat_hip.rendering import _reshape_view
        n_world = PAIR_SHARDS[WORLD]
        Nr = n_world[rank]
        g = torch.Generator().manual_seed(rank)
        radii = torch.randint(0, 50, (WORLD, Nr, 2), generator=g, dtype=torch.int32)
        fields = [torch.randn(WORLD, Nr, *sh, generator=g).requires_grad_(True)
                  for sh in ((2,), (), (3,), (), (3,))]
        wts = [torch.randn(1, sum(n_world), *f.shape[2:], generator=torch.Generator()
                           .manual_seed(10 + rank)) for f in fields]
        # the one field-major exchange
        out = gd.exchange_pairs(n_world, radii, *fields)
        sum((o * w).sum() for o, w in zip(out[1:], wts)).backward()
        fast = [out[0]] + [o.detach() for o in out[1:]]
        gfast = [f.grad.clone() for f in fields]
        for f in fields:
            f.grad = None
        # the generic path (rendering.py's C > 1 branch)
        splits, outs = [Nr] * WORLD, n_world
        (r2,) = gd.all_to_all_tensor_list(WORLD, [radii.flatten(0, 1)], splits=splits,
                                          output_splits=outs)
        parts = gd.all_to_all_tensor_list(WORLD, [f.flatten(0, 1) for f in fields],
                                          splits=splits, output_splits=outs)
        ref = [_reshape_view(1, r2, n_world)] + [_reshape_view(1, t, n_world) for t in parts]
        sum((o * w).sum() for o, w in zip(ref[1:], wts)).backward()
        ok = all(torch.equal(a, b.detach()) and a.is_contiguous() for a, b in zip(fast, ref))
        okg = all(torch.allclose(a, f.grad) for a, f in zip(gfast, fields))
        q.put((rank, (ok, okg, [tuple(t.shape) for t in fast])))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the test
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_exchange_pairs_matches_generic_exchange_gloo(world):
    """distributed.exchange_pairs (one field-major exchange, one camera per
    rank) gives the generic all_to_all_tensor_list + _reshape_view results,
    contiguous, and the same gradients, on 2 / 3 / 8 gloo ranks with uneven
    shards (every rank exchanging with several peers at 3 and 8)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pairs_worker, args=(r, port, q, world)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = sum(PAIR_SHARDS[world])
    for r in range(world):
        assert isinstance(res[r], tuple), res[r]
        ok, okg, shapes = res[r]
        assert ok and okg, (r, ok, okg)
        assert shapes == [(1, n, 2), (1, n, 2), (1, n), (1, n, 3), (1, n), (1, n, 3)]
