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
