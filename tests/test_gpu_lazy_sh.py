"""GPU: the lazy SH Adam (gsplat_hip_sh_colors_fwd_lazy, the lazy form of
gsplat_hip_sh_colors_bwd_adam(_dev), gsplat_hip_sh_lazy_flush; ABI 28).

Rows outside the view skip their zero-gradient Adam steps until they are
next visible or flushed.  The skipped steps are the same adam_update calls
in the same order, so:
* every step's colours equal those of the eagerly updated coefficients, bit
  for bit;
* after a flush the coefficients and both moments equal the eager
  sequence's, bit for bit -- also with step factors that change every step
  (a learning-rate schedule) and across the factor ring's wrap;
* the trainer with the lazy SH Adam tracks the trainer without it.
"""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def _case(N, seed=5):
    g = torch.Generator(device=DEV).manual_seed(seed)
    means = torch.randn(N, 3, device=DEV, generator=g) * 2
    vm = torch.eye(4, device=DEV)[None]
    vm[0, 2, 3] = 6.0
    sh0 = torch.randn(N, 1, 3, device=DEV, generator=g) * 0.3
    shN = torch.randn(N, 15, 3, device=DEV, generator=g) * 0.1
    return means, vm, sh0, shN, g


@pytest.mark.parametrize("R,steps", [(4096, 7), (4, 11)])
def test_lazy_sh_adam_is_exact(R, steps):
    """Random visibility per step (a row may stay out of view for several
    steps), per-step learning rates; R = 4 wraps the factor ring (the rows
    are flushed every R - 1 steps, as the trainer does)."""
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    from gsplat_hip.losses import adam_factors
    N = 3001
    means, vm, sh0, shN, g = _case(N)
    betas, eps = (0.9, 0.999), 1e-15
    radii_seq = [((torch.rand(1, N, device=DEV, generator=g) < 0.3).int() * 3)
                 for _ in range(steps)]
    vcol_seq = [torch.rand(1, N, 3, device=DEV, generator=g) - 0.5 for _ in range(steps)]
    lrs_seq = [(2.5e-3 * 0.97 ** t, 1.25e-4 * 0.97 ** t) for t in range(steps)]
    res = {}
    for lazy in (False, True):
        p0, pr = sh0.clone(), shN.clone()
        m0, v0 = torch.zeros_like(p0), torch.zeros_like(p0)
        mr, vr = torch.zeros_like(pr), torch.zeros_like(pr)
        last = torch.zeros(N, dtype=torch.int32, device=DEV)
        fac = torch.zeros(R, 4, device=DEV)
        vd = torch.empty(N, 3, device=DEV)
        hyper = torch.zeros(3, device=DEV)
        stepd = torch.zeros(1, dtype=torch.int64, device=DEV)
        cols = []
        flushed = 0
        for t in range(1, steps + 1):
            radii, vcol = radii_seq[t - 1], vcol_seq[t - 1]
            lr0, lrr = lrs_seq[t - 1]
            colors = torch.empty(1, N, 3, device=DEV)
            if lazy:
                if t - 1 - flushed >= R - 1:
                    _lib.call("gsplat_hip_sh_lazy_flush", N, _ptr(p0), _ptr(pr), _ptr(m0),
                              _ptr(v0), _ptr(mr), _ptr(vr), _ptr(last), _ptr(fac), R, t - 1,
                              0.9, 0.999, eps, _stream())
                    flushed = t - 1
                use_dev = t % 2 == 0  # the captured-step form on even steps
                stepd.fill_(t)
                _lib.call("gsplat_hip_sh_colors_fwd_lazy", 3, N, _ptr(means), _ptr(vm), _ptr(p0),
                          _ptr(pr), _ptr(radii), _ptr(colors), _ptr(m0), _ptr(v0), _ptr(mr),
                          _ptr(vr), _ptr(last), _ptr(fac), R, 0 if use_dev else t,
                          _ptr(stepd) if use_dev else None, 0.9, 0.999, eps, None, _stream())
                if use_dev:
                    (s0, ib), (sr, _) = adam_factors([lr0, lrr], betas, t)
                    hyper.copy_(torch.tensor([s0, sr, ib]))
                    _lib.call("gsplat_hip_sh_colors_bwd_adam_dev", 3, 1, N, _ptr(means),
                              _ptr(vm), _ptr(p0), _ptr(pr), _ptr(radii), _ptr(vcol), _ptr(vd),
                              _ptr(m0), _ptr(v0), _ptr(mr), _ptr(vr), _ptr(hyper),
                              ctypes.c_float(0.9), ctypes.c_float(0.999), ctypes.c_float(eps),
                              None, _ptr(last), _ptr(fac), R, _ptr(stepd), _stream())
                else:
                    _lib.call("gsplat_hip_sh_colors_bwd_adam", 3, 1, N, _ptr(means), _ptr(vm),
                              _ptr(p0), _ptr(pr), _ptr(radii), _ptr(vcol), _ptr(vd), _ptr(m0),
                              _ptr(v0), _ptr(mr), _ptr(vr), lr0, lrr, 0.9, 0.999, eps, t,
                              _ptr(last), _ptr(fac), R, _stream())
            else:
                _lib.call("gsplat_hip_sh_colors_fwd", 3, 1, N, N, 16, _ptr(means), _ptr(vm),
                          _ptr(p0), _ptr(pr), _ptr(radii), _ptr(colors), _stream())
                _lib.call("gsplat_hip_sh_colors_bwd_adam", 3, 1, N, _ptr(means), _ptr(vm),
                          _ptr(p0), _ptr(pr), _ptr(radii), _ptr(vcol), _ptr(vd), _ptr(m0),
                          _ptr(v0), _ptr(mr), _ptr(vr), lr0, lrr, 0.9, 0.999, eps, t, None,
                          None, 0, _stream())
            cols.append(colors.clone())
        if lazy:
            _lib.call("gsplat_hip_sh_lazy_flush", N, _ptr(p0), _ptr(pr), _ptr(m0), _ptr(v0),
                      _ptr(mr), _ptr(vr), _ptr(last), _ptr(fac), R, steps, 0.9, 0.999, eps,
                      _stream())
            assert int(last.min()) == int(last.max()) == steps
        torch.cuda.synchronize()
        res[lazy] = (cols, (p0, pr, m0, v0, mr, vr))
    for a, b in zip(res[False][0], res[True][0]):
        assert torch.equal(a, b)
    for a, b in zip(res[False][1], res[True][1]):
        assert torch.equal(a, b)


def test_trainer_lazy_sh_tracks_eager(monkeypatch):
    """Trainer with and without the lazy SH Adam over 6 steps of a 3-camera
    pool (part of the scene out of view each step): after Trainer.sync the
    parameters and the SH moments agree (the rasterizer's float atomics
    make two runs differ in the last bits)."""
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(root, "tests", "golden", "garden_scene.npz"), scene_grid=1)
    means, rgbs = means[::8].contiguous(), rgbs[::8].contiguous()
    W, H = 320, 240
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=3)
    out = {}
    for lazy in ("0", "1"):
        monkeypatch.setenv("GSPLAT_HIP_SH_LAZY", lazy)
        tr = Trainer(means, rgbs, vm, K, W, H, device=DEV, graph=False, max_steps=100)
        assert (tr.sh_lazy is not None) == (lazy == "1")
        for it in range(6):
            tr.step(it)
        tr.sync()
        names = list(tr.params)
        out[lazy] = ({k: p.detach().clone() for k, p in tr.params.items()},
                     [tr.opt.exp_avg[names.index(k)].clone() for k in ("sh0", "shN")])
    for k in out["0"][0]:
        torch.testing.assert_close(out["1"][0][k], out["0"][0][k], rtol=1e-3, atol=1e-5)
    for a, b in zip(out["0"][1], out["1"][1]):
        torch.testing.assert_close(b, a, rtol=1e-2, atol=1e-6)
