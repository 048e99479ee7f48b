"""GPU: the trainer's visible_adam option (simple_trainer.py:263-266,782-797):
SelectiveAdam -- the reference's Adam kernel, no bias correction, applied
only to the rows of the Gaussians the step's camera sees, (radii > 0).any(0)
-- through gsplat_hip_selective_adam, one launch per parameter group."""

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
