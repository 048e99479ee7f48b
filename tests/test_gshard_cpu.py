"""CPU: the Gaussian-sharded trainer's host logic (Trainer(gaussian_shard=True);
the render itself needs the GPU, tests/test_gpu_gshard.py).

* rank r's Gaussians are the one-GPU scene's [r::world], initialised as a
  whole first (simple_trainer.py:221-229), with the batch learning-rate
  scaling of world cameras per step (:261-277);
* the camera schedule every rank derives for step it -- rank r renders
  (it * world + r) % n -- is the same list on every rank.
"""

import math
import os

import torch

from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene():
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=1)
    means, rgbs = means[::16].contiguous(), rgbs[::16].contiguous()
    vm, K = camera_pool(vms, Ks, sw, sh_, 64, 48, n=5)
    return means, rgbs, vm, K


def test_shards_are_slices_of_the_whole_scene():
    means, rgbs, vm, K = _scene()
    N = means.shape[0]
    whole = Trainer(means, rgbs, vm, K, 64, 48, device="cpu", fused=False)
    for world in (2, 3):
        total = 0
        for rank in range(world):
            tr = Trainer(means, rgbs, vm, K, 64, 48, device="cpu", fused=False,
                         world_size=world, rank=rank, gaussian_shard=True)
            assert tr.gshard and not tr.sharded
            assert tr._n_world == [len(range(r, N, world)) for r in range(world)]
            for k, p in tr.params.items():
                assert torch.equal(p.detach(), whole.params[k].detach()[rank::world]), k
            assert tr.grad2d.shape == (tr._n_world[rank],)
            for lr, lr1 in zip(tr.lrs, whole.lrs):
                assert math.isclose(lr, lr1 * math.sqrt(world), rel_tol=1e-12)
            total += tr.params["means"].shape[0]
        assert total == N


def test_world_camera_schedule_agrees_across_ranks():
    means, rgbs, vm, K = _scene()
    world, n = 3, len(vm)
    trs = [Trainer(means, rgbs, vm, K, 64, 48, device="cpu", fused=False, world_size=world,
                   rank=r, gaussian_shard=True) for r in range(world)]
    for it in range(7):
        lists = []
        for tr in trs:
            ci = tr.camera_index(it)
            vms, ks = tr.world_cameras(ci)
            want = [(it * world + r) % n for r in range(world)]
            assert torch.equal(vms, vm[want]) and torch.equal(ks, K[want])
            lists.append(vms)
        assert all(torch.equal(lists[0], x) for x in lists[1:])
    # evaluation: every rank renders the same camera
    vms, _ = trs[1].world_cameras(2, world_ci=[2] * world)
    assert torch.equal(vms, vm[[2, 2, 2]])


def test_emulated_exchange_rows():
    """bench.py --gshard-emulate: a recording render keeps the rows a peer
    sends to rank 0 (its first block) and stops at its float exchange; rank
    0's exchanges then take those rows in the peers' places (forward) and its
    own gradient block in every peer's place (backward)."""
    from gsplat_hip import distributed as gdist
    emu = gdist.Emulation(3)
    n = [4, 4, 3]  # Gaussians per rank; one camera per rank

    def peer_render(j):
        radii = torch.arange(3 * n[j], dtype=torch.int32).view(3 * n[j], 1) + 100 * j
        rows = torch.arange(3 * n[j] * 2, dtype=torch.float32).view(3 * n[j], 2) + 1000 * j
        splits = [n[j]] * 3  # camera-major blocks: camera r's rows go to rank r
        outs = [n[r] for r in range(3)]
        gdist._all_to_all_rows(radii, splits, outs)
        gdist._all_to_all_rows(rows, splits, outs)
        raise AssertionError("a recording render stops at its float exchange")

    prev = gdist.EMULATION
    gdist.EMULATION = emu
    try:
        for j in (1, 2):
            emu.record(j, lambda: peer_render(j))
        assert gdist.rank_world() == (0, 3)
        rows0 = torch.arange(3 * n[0] * 2, dtype=torch.float32).view(3 * n[0], 2)
        got = gdist._all_to_all_rows(rows0, [n[0]] * 3, n)
        assert torch.equal(got[:4], rows0[:4])
        for j in (1, 2):
            want = torch.arange(3 * n[j] * 2, dtype=torch.float32).view(3 * n[j], 2)[:n[j]] + 1000 * j
            assert torch.equal(got[sum(n[:j]):sum(n[:j + 1])], want)
        r0 = gdist._all_to_all_rows(torch.zeros(3 * n[0], 1, dtype=torch.int32), [n[0]] * 3, n)
        assert torch.equal(r0[4:8].flatten(), torch.arange(4, dtype=torch.int32) + 100)
        grad = torch.randn(sum(n), 2)
        back = gdist._all_to_all_rows(grad, n, [n[0]] * 3, backward=True)
        assert torch.equal(back, grad[:4].repeat(3, 1))
    finally:
        gdist.EMULATION = prev
