"""GPU checks of the training-step kernels against fp32 torch references:
fused SSIM+L1 (vs the conv formulation of fused_ssim's algorithm, autograd)
and the one-launch Adam (vs torch.optim.Adam)."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("B,H,W,C", [(1, 64, 80, 3), (2, 37, 131, 3), (1, 11, 11, 1), (1, 270, 480, 3)])
def test_ssim_l1_matches_torch(B, H, W, C):
    from gsplat_hip.losses import ssim_and_l1
    from gsplat_hip.train_step import ssim
    g = torch.Generator(device="cuda").manual_seed(H * W)
    img = torch.rand(B, H, W, C, device="cuda", generator=g).requires_grad_(True)
    gt = torch.rand(B, H, W, C, device="cuda", generator=g)
    s, l1 = ssim_and_l1(img, gt)
    img_r = img.detach().clone().requires_grad_(True)
    s_r = ssim(img_r.permute(0, 3, 1, 2), gt.permute(0, 3, 1, 2))
    l1_r = (img_r - gt).abs().mean()
    torch.testing.assert_close(s, s_r, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(l1, l1_r, rtol=1e-5, atol=1e-6)
    (0.3 * s + 0.7 * l1).backward()
    (0.3 * s_r + 0.7 * l1_r).backward()
    torch.testing.assert_close(img.grad, img_r.grad, rtol=1e-3, atol=1e-8)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("B,H,W,C,lam", [(1, 64, 80, 3, 0.2), (2, 37, 131, 3, 0.5),
                                         (1, 1080, 1920, 3, 0.2), (1, 11, 11, 1, 0.3),
                                         (3, 45, 33, 1, 0.2), (1, 100, 12, 3, 0.8)])
def test_l1_ssim_loss_matches_torch(B, H, W, C, lam, fused):
    """The one-launch-pair loss (and the one-pass fused loss + gradient)
    equals the simple_trainer.py:642-646 formula evaluated with torch ops on
    the conv SSIM."""
    from gsplat_hip.losses import l1_ssim_loss
    from gsplat_hip.train_step import ssim
    g = torch.Generator(device="cuda").manual_seed(W + C)
    img = torch.rand(B, H, W, C, device="cuda", generator=g).requires_grad_(True)
    gt = torch.rand(B, H, W, C, device="cuda", generator=g)
    loss = l1_ssim_loss(img, gt, lam, fused=fused)
    img_r = img.detach().clone().requires_grad_(True)
    s_r = ssim(img_r.permute(0, 3, 1, 2), gt.permute(0, 3, 1, 2))
    loss_r = (img_r - gt).abs().mean() * (1 - lam) + (1 - s_r) * lam
    assert loss.dim() == 0
    torch.testing.assert_close(loss, loss_r, rtol=1e-4, atol=1e-5)
    (2.5 * loss).backward()
    (2.5 * loss_r).backward()
    torch.testing.assert_close(img.grad, img_r.grad, rtol=1e-3, atol=1e-9)


@pytest.mark.parametrize("H,W,ring", [(64, 80, False), (1080, 1920, False), (37, 131, True)])
def test_fused_loss_reads_rgbd_render_in_place(H, W, ring):
    """The fused loss over the colour channels of an RGB+D render read in
    place (x_stride 4, the 2DGS trainer's loss) equals the loss of the
    contiguous colour copy, value and gradient, to float rounding (the
    in-place kernel blocks its vertical pass by 2 rows, not 4: at 128 VGPRs
    the 4-row form spilled 25 of them with the strided reads); the depth
    channel's gradient is exactly zero (no slice copy, no zero-filled
    gradient image)."""
    from gsplat_hip.losses import ONE_GRAD, l1_ssim_loss
    import gsplat_hip.losses as L
    g = torch.Generator(device="cuda").manual_seed(H + W)
    rgbd = torch.rand(1, H, W, 4, device="cuda", generator=g)
    gt = torch.rand(3, H, W, 3, device="cuda", generator=g)
    idx = torch.tensor([1], device="cuda")
    kw = {}
    if ring:
        kw = dict(gt_index=idx, _out_ring=(torch.zeros(8, device="cuda"),
                                          torch.ones(1, dtype=torch.int64, device="cuda")))
    target = gt if ring else gt[1:2].contiguous()
    a = rgbd.clone().requires_grad_(True)
    b = rgbd[..., :3].contiguous().requires_grad_(True)
    la = l1_ssim_loss(a, target, 0.2, fused=True, _channels=3, **kw)
    lb = l1_ssim_loss(b, target, 0.2, fused=True, **kw)
    torch.testing.assert_close(la, lb, rtol=1e-6, atol=0)
    la.backward()
    lb.backward()
    assert a.grad.shape == (1, H, W, 4)
    torch.testing.assert_close(a.grad[..., :3], b.grad, rtol=1e-5,
                               atol=1e-6 * float(b.grad.abs().max()))
    assert torch.equal(a.grad[..., 3], torch.zeros_like(a.grad[..., 3]))


def test_fused_loss_matches_two_pass_on_renders():
    """Fused vs two-pass loss on a smooth, correlated image pair (a render
    and a shifted copy, as in training): same loss, same gradient up to the
    summation order of the blurs, and a second backward gives the same."""
    from gsplat_hip.losses import l1_ssim_loss
    g = torch.Generator(device="cuda").manual_seed(4)
    base = torch.nn.functional.avg_pool2d(torch.rand(1, 3, 300, 420, device="cuda",
                                                     generator=g), 5, 1, 2)
    img = base[:, :, :, 2:].permute(0, 2, 3, 1).contiguous()
    gt = base[:, :, :, :-2].permute(0, 2, 3, 1).contiguous()
    a = img.clone().requires_grad_(True)
    b = img.clone().requires_grad_(True)
    la = l1_ssim_loss(a, gt, 0.2, fused=True)
    lb = l1_ssim_loss(b, gt, 0.2, fused=False)
    torch.testing.assert_close(la, lb, rtol=1e-5, atol=1e-6)
    (3.0 * la).backward(retain_graph=True)
    (3.0 * lb).backward()
    # near-cancelling pixels: absolute bound relative to the gradient's scale
    scale = float(b.grad.abs().max())
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-4 * scale)
    g1 = a.grad.clone()
    a.grad = None
    (3.0 * la).backward()
    assert torch.equal(a.grad, g1)


def test_fused_adam_matches_torch():
    from gsplat_hip.losses import FusedAdam
    torch.manual_seed(0)
    shapes = [(1001, 3), (1001, 4), (1001,), (1001, 15, 3)]
    lrs = [1.6e-4, 1e-3, 5e-2, 2.5e-3 / 20]
    ps = [torch.randn(s, device="cuda") for s in shapes]
    qs = [p.clone().requires_grad_(True) for p in ps]
    ps = [p.requires_grad_(True) for p in ps]
    kw = dict(betas=(0.9, 0.999), eps=1e-15)
    ref = torch.optim.Adam([{"params": [q], "lr": lr} for q, lr in zip(qs, lrs)], **kw)
    mine = FusedAdam(ps, lrs, **kw)
    for it in range(5):
        gs = [torch.randn_like(p) for p in ps]
        for p, q, gr in zip(ps, qs, gs):
            p.grad = gr.clone()
            q.grad = gr.clone()
        ref.step()
        mine.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_activate_matches_torch_exactly():
    """exp / sigmoid and their VJPs in one launch each way equal torch's."""
    from gsplat_hip.strategy import activate
    g = torch.Generator(device="cuda").manual_seed(5)
    ls = (torch.randn(10007, 3, device="cuda", generator=g) * 3).requires_grad_(True)
    lg = (torch.randn(10007, device="cuda", generator=g) * 6).requires_grad_(True)
    s, o = activate(ls, lg)
    ls_r = ls.detach().clone().requires_grad_(True)
    lg_r = lg.detach().clone().requires_grad_(True)
    s_r, o_r = torch.exp(ls_r), torch.sigmoid(lg_r)
    assert torch.equal(s, s_r) and torch.equal(o, o_r)
    vs = torch.randn_like(s)
    vo = torch.randn_like(o)
    ((s * vs).sum() + (o * vo).sum()).backward()
    ((s_r * vs).sum() + (o_r * vo).sum()).backward()
    assert torch.equal(ls.grad, ls_r.grad) and torch.equal(lg.grad, lg_r.grad)


@pytest.mark.parametrize("C,N", [(1, 5003), (3, 5003), (3, 5004)])
def test_update_state_matches_torch(C, N):
    """DefaultStrategy._update_state (default.py:213-262) with torch ops vs the
    one-launch HIP version, over two steps (accumulation)."""
    from gsplat_hip.strategy import update_state_
    W, H = 640, 480
    g = torch.Generator(device="cuda").manual_seed(C)
    grad2d = torch.zeros(N, device="cuda")
    count = torch.zeros(N, device="cuda")
    g_r, c_r = grad2d.clone(), count.clone()
    for _ in range(2):
        m2g = torch.randn(C, N, 2, device="cuda", generator=g) * 1e-3
        radii = torch.randint(-1, 3, (C, N), device="cuda", generator=g, dtype=torch.int32)
        update_state_(grad2d, count, m2g, radii, W, H, C)
        grads = m2g.clone()
        grads[..., 0] *= W / 2.0 * C
        grads[..., 1] *= H / 2.0 * C
        sel = radii > 0
        ids = torch.where(sel)[1]
        g_r.index_add_(0, ids, grads[sel].norm(dim=-1))
        c_r.index_add_(0, ids, torch.ones_like(ids, dtype=torch.float32))
    torch.testing.assert_close(grad2d, g_r, rtol=1e-6, atol=0)
    assert torch.equal(count, c_r)


def _small_scene(n_cams=4, W=320, H=240):
    import os as _os
    from gsplat_hip.train_step import camera_pool, load_garden_scene
    root = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        _os.path.join(root, "tests", "golden", "garden_scene.npz"), scene_grid=1)
    means, rgbs = means[::8].contiguous(), rgbs[::8].contiguous()
    vm, K = camera_pool(vms, Ks, sw, sh_, W, H, n=n_cams)
    return means, rgbs, vm, K, W, H


def thr_first(tr):
    from gsplat_hip import _wrapper
    with _wrapper.fwd_split(tr.split_div):
        colors, _, meta = tr.render(tr.camera_index(0), tr.sh_degree_at(0))
        return _wrapper.fwd_split_threshold(meta["flatten_ids"].numel())


def test_trainer_tunes_split_divisor_from_termination():
    """Trainer._tune_split: before the first step, the forward's n_eff /
    n_isects (forward_termination_ratio, the bench's formula) picks the split
    threshold's divisor: 1100 above 0.75, else 550.  The divisor is the
    trainer's own: inside its renders the library reports it, outside the
    process-wide value is left as it was.  The ratio is checked against a
    direct per-tile evaluation."""
    from gsplat_hip import _lib, _wrapper
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    try:
        before = _lib.query("gsplat_hip_set_fwd_split_div", 777)  # a sentinel
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", max_steps=100)
        tr.step(0)
        r = tr.term_ratio
        assert 0.0 < r <= 1.0
        assert tr.split_div == (1100 if r > 0.75 else 550)
        # the forward variant: decided once from the first render's largest tile
        with _wrapper.fwd_split(tr.split_div):
            thr = _wrapper.fwd_split_threshold(1)
        assert tr.split_launch in (0, 1) and thr >= 2048
        old_thr = _lib.query("gsplat_hip_set_fwd_split_threshold", -1)
        assert old_thr == -1, old_thr  # not leaked
        assert tr.split_threshold == (thr_first(tr) if tr.split_launch else 0)
        assert _lib.query("gsplat_hip_set_fwd_split_div", 777) == 777  # not leaked
        with _wrapper.fwd_split(tr.split_div):
            assert _lib.query("gsplat_hip_set_fwd_split_div", tr.split_div) == tr.split_div
        assert _lib.query("gsplat_hip_set_fwd_split_div", before) == 777
        # direct: per tile, isects up to the tile's largest last id + 1
        colors, _, meta = tr.render(tr.camera_index(0), tr.sh_degree_at(0))
        r2 = _wrapper.forward_termination_ratio(colors, meta, W, H)
        node = colors.grad_fn
        while type(node).__name__ != "_RasterizeToPixelsBackward":
            node = node.next_functions[0][0]
        last = node.saved_tensors[9][0].cpu().numpy()
        offs = meta["isect_offsets"].flatten().cpu().numpy().astype(np.int64)
        n = meta["flatten_ids"].numel()
        ts, tw, th = meta["tile_size"], meta["tile_width"], meta["tile_height"]
        n_eff = 0
        for t in range(tw * th):
            y, x = divmod(t, tw)
            end = offs[t + 1] if t + 1 < len(offs) else n
            blk = last[y * ts:(y + 1) * ts, x * ts:(x + 1) * ts]
            if end > offs[t]:
                n_eff += max(0, min(end, int(blk.max()) + 1) - offs[t])
        assert abs(r2 - n_eff / n) < 1e-9, (r2, n_eff / n)
    finally:
        _lib.query("gsplat_hip_set_fwd_split_div", 0)


@pytest.mark.parametrize("sharded", [False, True])
def test_trainer_densification_schedule(sharded):
    """The simple_trainer default schedule on the HIP path (compressed in
    time): SfM init with knn scales, SH degree schedule, means LR decay,
    refine every 2 steps and opacity reset every 5.  Every refine rebuilds the
    parameters and the optimizer state consistently (sizes; the decisions
    themselves are pinned by test_gpu_strategy.py) and training keeps going,
    with the fused optimizer and with the sharded one on one RCCL rank (its
    state gathered, compacted and re-sharded).  The multi-rank statistics sum
    and shared noise: tests/test_distributed.py (gloo)."""
    import torch.distributed as dist
    own_pg = sharded and not dist.is_initialized()
    if own_pg:
        import os as _os
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        _os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        _densification_schedule(sharded)
    finally:
        if own_pg:
            dist.destroy_process_group()


def _densification_schedule(sharded):
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    cfg = DefaultStrategyConfig(refine_start_iter=1, refine_every=2, reset_every=5)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", strategy=cfg, sh_degree_interval=2,
                 max_steps=100, init="sfm", sharded_optimizer=sharded)
    losses = []
    for it in range(7):
        losses.append(float(tr.step(it)))
        n = tr.params["means"].shape[0]
        for k, p in tr.params.items():
            assert p.shape[0] == n, k
        for k, (m, v) in tr.moments().items():
            assert m.shape == tr.params[k].shape and v.shape == tr.params[k].shape, k
        assert tr.grad2d.numel() == n and tr.count.numel() == n
        if it == 5:  # reset_every: opacities clamped to logit(0.01), moments zero
            tr.sync()
            lim = float(torch.logit(torch.tensor(0.01)))
            assert float(tr.params["opacities"].max()) <= lim + 1e-6
            assert float(tr.moments()["opacities"][0].abs().max()) == 0.0
    assert [r[0] for r in tr.refine_log] == [2, 4, 6], tr.refine_log
    assert all(math.isfinite(x) for x in losses), losses
    n0 = means.shape[0]
    assert tr.refine_log[0][4] == n0 + tr.refine_log[0][1] + tr.refine_log[0][2] \
        - tr.refine_log[0][3], tr.refine_log
    assert tr.refine_log[0][1] + tr.refine_log[0][2] > 0  # random targets: something grows
    tr.sync()


def test_trainer_evaluate_psnr_ssim():
    """Trainer.evaluate (simple_trainer.py:854-932 metrics): PSNR of the
    clamped render equals -10 log10(MSE) computed here, SSIM is the fused
    valid SSIM; a target equal to the render gives SSIM 1 and a huge PSNR."""
    from gsplat_hip.losses import ssim_and_l1
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda")
    for it in range(3):
        tr.step(it)
    m = tr.evaluate([0, 2])
    with torch.no_grad():
        ps, ss = [], []
        for ci in (0, 2):
            c, _, _ = tr.render(ci)
            c = c.clamp(0, 1)
            gt = tr.targets[ci:ci + 1]
            ps.append(float(-10 * torch.log10(((c - gt) ** 2).mean())))
            ss.append(float(ssim_and_l1(c, gt)[0]))
    assert m["num_images"] == 2
    assert abs(m["psnr"] - sum(ps) / 2) < 1e-4 and abs(m["ssim"] - sum(ss) / 2) < 1e-5
    with torch.no_grad():
        c, _, _ = tr.render(1)
    same = tr.evaluate(viewmats=vm[1:2], Ks=K[1:2], images=c.clamp(0, 1).cpu())
    assert same["ssim"] > 0.999 and same["psnr"] > 60


@pytest.mark.parametrize("degree", [3, 1])
def test_sh_adam_in_backward_is_exact(degree):
    """The SH-colour backward with the coefficients' Adam step fused in
    (gsplat_hip_sh_colors_bwd_adam) leaves the coefficients and moments
    bit-identical to the plain backward + FusedAdam, over several steps, and
    returns the same means gradient; invisible rows get their zero-gradient
    Adam update too.  Below degree 3 the armed backward declines (unfused)."""
    from gsplat_hip import _wrapper
    from gsplat_hip.losses import FusedAdam
    g = torch.Generator(device="cuda").manual_seed(5)
    N = 3001  # a last wave of 57 rows: scalar tails of the float4 walk
    means = torch.randn(N, 3, device="cuda", generator=g) * 2
    vm = torch.eye(4, device="cuda")[None]
    vm[0, 2, 3] = 6.0
    radii = (torch.rand(1, N, device="cuda", generator=g) > 0.4).int() * 3
    sh0 = torch.randn(N, 1, 3, device="cuda", generator=g) * 0.3
    shN = torch.randn(N, 15, 3, device="cuda", generator=g) * 0.1
    ws = [torch.rand(1, N, 3, device="cuda", generator=g) - 0.5 for _ in range(4)]
    res = []
    for fused in (False, True):
        p0 = sh0.clone().requires_grad_(True)
        p1 = shN.clone().requires_grad_(True)
        mm = means.clone().requires_grad_(True)
        opt = FusedAdam([p0, p1], [2.5e-3, 2.5e-3 / 20], betas=(0.9, 0.999), eps=1e-15)
        gm = []
        for it in range(4):
            fa = fusion = None
            if fused:
                fa = _wrapper.ShAdamInBackward(p0.data, p1.data, opt.exp_avg[0], opt.exp_avg_sq[0],
                                               opt.exp_avg[1], opt.exp_avg_sq[1], opt.lrs[0],
                                               opt.lrs[1], opt.betas, opt.eps, opt.step_count + 1)
                fusion = _wrapper.StepFusion(sh_adam=fa)
            colors = _wrapper.sh_colors(degree, mm, vm, (p0, p1), radii, fusion=fusion)
            (colors * ws[it]).sum().backward()
            if fused and degree == 3:
                assert fa.applied and p0.grad is None and p1.grad is None
                opt.step(skip=(0, 1))
            else:  # lower degrees: the armed backward falls back to the unfused one
                assert fa is None or not fa.applied
                opt.step()
            opt.zero_grad()
            gm.append(mm.grad.clone())
            mm.grad = None
        torch.cuda.synchronize()
        res.append((p0.detach().clone(), p1.detach().clone(), *opt.exp_avg, *opt.exp_avg_sq, *gm))
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_adam_gradient_transforms_are_exact():
    """gsplat_hip_adam_step_ex's in-register gradients (sum, exp VJP, sigmoid
    VJP) give the same bits as forming them first (activate_bwd's formulas)
    and stepping FusedAdam on the result."""
    from gsplat_hip.losses import FusedAdam
    torch.manual_seed(1)
    N = 4099  # scalar tails
    shapes = [(N, 3), (N, 4), (N, 3), (N,)]
    base = [torch.randn(s, device="cuda") for s in shapes]
    lrs = [1.6e-4, 1e-3, 5e-3, 5e-2]
    res = []
    for fused in (False, True):
        ps = [b.clone().requires_grad_(True) for b in base]
        opt = FusedAdam(ps, lrs, betas=(0.9, 0.999), eps=1e-15)
        for it in range(3):
            g = torch.Generator(device="cuda").manual_seed(10 + it)
            ga, gb = (torch.randn(N, 3, device="cuda", generator=g) for _ in range(2))
            gq = torch.randn(N, 4, device="cuda", generator=g)
            vs = torch.randn(N, 3, device="cuda", generator=g)
            vo = torch.randn(N, device="cuda", generator=g)
            s_act = torch.exp(ps[2].detach())
            o_act = torch.sigmoid(ps[3].detach())
            if fused:
                ps[0].grad, ps[1].grad = ga, gq
                opt.step(xform={0: (ga, gb, 1), 2: (vs, s_act, 2), 3: (vo, o_act, 3)})
            else:
                ps[0].grad, ps[1].grad = ga + gb, gq
                ps[2].grad, ps[3].grad = vs * s_act, vo * (1 - o_act) * o_act
                opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        res.append([p.detach().clone() for p in ps] + opt.exp_avg + opt.exp_avg_sq)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_trainer_geometry_fusion_close(monkeypatch):
    """The trainer with the activation VJPs / means sum folded into the
    geometry update (GSPLAT_HIP_GEOM_FUSE=1) tracks the unfused trainer (the
    rasterizer's backward atomics make two runs differ in the last bits)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    out = {}
    for f in ("0", "1"):
        monkeypatch.setenv("GSPLAT_HIP_GEOM_FUSE", f)
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda")
        assert tr.geom_fuse == (f == "1")
        losses = [float(tr.step(it)) for it in range(5)]
        out[f] = (losses, {k: p.detach().clone() for k, p in tr.params.items()})
    for a, b in zip(out["0"][0], out["1"][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-7, (out["0"][0], out["1"][0])
    for k in out["0"][1]:
        torch.testing.assert_close(out["1"][1][k], out["0"][1][k], rtol=1e-3, atol=1e-5)


def test_fused_loss_constant_seed_skips_scaling_exactly():
    """Seeded with losses.ONE_GRAD, the fused loss's backward returns its
    unit gradient as is: the same bits as the scaled path with a 1.0 seed."""
    from gsplat_hip import losses
    g = torch.Generator(device="cuda").manual_seed(8)
    img = torch.rand(1, 70, 90, 3, device="cuda", generator=g)
    gt = torch.rand(1, 70, 90, 3, device="cuda", generator=g)
    a = img.clone().requires_grad_(True)
    b = img.clone().requires_grad_(True)
    old = losses.ONE_GRAD
    losses.ONE_GRAD = torch.ones((), device="cuda")
    try:
        torch.autograd.backward(losses.l1_ssim_loss(a, gt, 0.2, fused=True), losses.ONE_GRAD)
    finally:
        seed, losses.ONE_GRAD = losses.ONE_GRAD, old
    torch.autograd.backward(losses.l1_ssim_loss(b, gt, 0.2, fused=True),
                            torch.ones((), device="cuda"))
    assert torch.equal(a.grad, b.grad)
    assert float(seed) == 1.0


def test_fusion_context_is_per_render():
    """The fused optimizer work travels with the StepFusion handed to one
    forward: a second render in between (no fusion object) keeps ordinary
    gradients, and the fused node still applies its Adam step exactly once."""
    from gsplat_hip import _wrapper
    from gsplat_hip.losses import FusedAdam
    g = torch.Generator(device="cuda").manual_seed(7)
    N = 777
    means = (torch.randn(N, 3, device="cuda", generator=g) * 2).requires_grad_(True)
    vm = torch.eye(4, device="cuda")[None]
    vm[0, 2, 3] = 6.0
    radii = (torch.rand(1, N, device="cuda", generator=g) > 0.3).int() * 3
    p0 = (torch.randn(N, 1, 3, device="cuda", generator=g) * 0.3).requires_grad_(True)
    p1 = (torch.randn(N, 15, 3, device="cuda", generator=g) * 0.1).requires_grad_(True)
    w = torch.rand(1, N, 3, device="cuda", generator=g) - 0.5
    opt = FusedAdam([p0, p1], [2.5e-3, 1.25e-4], eps=1e-15)
    fa = _wrapper.ShAdamInBackward(p0.data, p1.data, opt.exp_avg[0], opt.exp_avg_sq[0],
                                   opt.exp_avg[1], opt.exp_avg_sq[1], opt.lrs[0], opt.lrs[1],
                                   opt.betas, opt.eps, 1)
    fusion = _wrapper.StepFusion(sh_adam=fa, geom=True)
    c_fused = _wrapper.sh_colors(3, means, vm, (p0, p1), radii, fusion=fusion)
    before = p0.detach().clone()
    # an unrelated render + backward between the fused forward and its backward
    other = _wrapper.sh_colors(3, means, vm, (p0, p1), radii)
    (other * w).sum().backward()
    assert p0.grad is not None and p1.grad is not None and means.grad is not None
    assert not fa.applied and fusion.v_dirs is None
    assert torch.equal(p0.detach(), before)
    g_other = (p0.grad.clone(), means.grad.clone())
    p0.grad = p1.grad = means.grad = None
    (c_fused * w).sum().backward()
    assert fa.applied and p0.grad is None and p1.grad is None
    assert means.grad is None and fusion.v_dirs is not None  # handed to the geometry update
    torch.testing.assert_close(fusion.v_dirs, g_other[1], rtol=0, atol=0)
    assert not torch.equal(p0.detach(), before)  # updated in place, once


def test_trainer_regulariser_with_fusions_matches_unfused(monkeypatch):
    """simple_trainer's opacity / scale regularisers (terms on the raw
    parameters, simple_trainer.py:671-681) reach .grad outside the fused
    nodes; the fused geometry update adds them as extra terms, so the fused
    trainer tracks the unfused one (nothing is dropped)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    out = {}
    for f in ("0", "1"):
        monkeypatch.setenv("GSPLAT_HIP_GEOM_FUSE", f)
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", opacity_reg=0.5, scale_reg=5.0)
        assert tr.geom_fuse == (f == "1")
        losses = [float(tr.step(it)) for it in range(4)]
        out[f] = (losses, {k: p.detach().clone() for k, p in tr.params.items()})
    for a, b in zip(out["0"][0], out["1"][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-7, (out["0"][0], out["1"][0])
    for k in out["0"][1]:
        torch.testing.assert_close(out["1"][1][k], out["0"][1][k], rtol=1e-3, atol=1e-5)
    # and the regulariser changes the result (it is not silently dropped)
    monkeypatch.setenv("GSPLAT_HIP_GEOM_FUSE", "1")
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda")
    for it in range(4):
        tr.step(it)
    assert not torch.allclose(tr.params["opacities"], out["1"][1]["opacities"], rtol=0, atol=1e-6)


def test_trainer_tracks_screen_radii_for_scale2d_refine():
    """refine_scale2d_stop_iter > 0 (default.py:235-262, 283-284, 325-326):
    the trainer keeps state["radii"] (max screen radius / max(W, H)), hands
    it to the refine before the stop step and restarts it after a refine;
    the kernel's use of it is pinned by the densify_scale2d golden
    (test_gpu_strategy.py)."""
    from gsplat_hip.densify import DefaultStrategyConfig
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    cfg = DefaultStrategyConfig(refine_start_iter=1, refine_every=2, reset_every=100,
                                refine_scale2d_stop_iter=3)
    tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", strategy=cfg, init="sfm")
    assert cfg.key_for_gradient == "means2d" and tr.strategy is not cfg  # caller's config untouched
    tr.step(0)
    meta = tr.last_meta
    exp = meta["radii"][0].float() / float(max(W, H))
    torch.testing.assert_close(tr.radii2d, exp, rtol=0, atol=0)
    tr.step(1)
    n_before = tr.params["means"].shape[0]
    tr.step(2)  # refine with the screen-size split / prune
    assert [r[0] for r in tr.refine_log] == [2]
    n_after = tr.params["means"].shape[0]
    assert n_after == tr.refine_log[0][-1] and tr.radii2d.shape == (n_after,)
    assert float(tr.radii2d.abs().sum()) == 0.0
    # splits happened (the screen-size rule adds every Gaussian over 5 % of the image)
    assert tr.refine_log[0][2] > 0 and n_before > 0
    for it in range(3, 6):
        assert math.isfinite(float(tr.step(it)))


@pytest.mark.parametrize("dev_factors", [False, True])
def test_projection_backward_adam_is_exact(dev_factors):
    """gsplat_hip_projection_bwd_adam (the geometry groups' Adam inside the
    projection backward) gives the same bits as the projection backward that
    stores the gradients, then FusedAdam with the trainer's in-register
    transforms (means + v_dirs, exp VJP, sigmoid VJP) -- host and device
    factor forms, invisible Gaussians and a ragged N included."""
    import ctypes
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    from gsplat_hip.losses import FusedAdam, adam_factors
    g = torch.Generator().manual_seed(3)
    N, W, H = 3001, 320, 240
    means = (torch.randn(N, 3, generator=g) * 0.8 + torch.tensor([0, 0, 4.0])).cuda()
    logs = torch.log(torch.rand(N, 3, generator=g) * 0.05 + 0.005).cuda()
    quats = torch.nn.functional.normalize(torch.randn(N, 4, generator=g), dim=-1).cuda()
    logit = torch.randn(N, generator=g).cuda()
    vm = torch.eye(4)[None].cuda()
    K = torch.tensor([[[300.0, 0, 160], [0, 300.0, 120], [0, 0, 1]]]).cuda()
    lrs = [1.6e-4, 5e-3, 1e-3, 5e-2]
    res = []
    for fused in (False, True):
        ps = [t.clone() for t in (means, logs, quats, logit)]
        opt = FusedAdam([torch.nn.Parameter(p) for p in ps], lrs, betas=(0.9, 0.999), eps=1e-15)
        ps = [p.data for p in opt.params]
        for it in range(3):
            gg = torch.Generator(device="cuda").manual_seed(20 + it)
            scales = torch.exp(ps[1])
            opac = torch.sigmoid(ps[3])
            radii = torch.empty(1, N, dtype=torch.int32, device="cuda")
            m2 = torch.empty(1, N, 2, device="cuda")
            dep = torch.empty(1, N, device="cuda")
            con = torch.empty(1, N, 3, device="cuda")
            _lib.call("gsplat_hip_projection_fwd", 1, N, _ptr(ps[0]), _ptr(ps[2]), _ptr(scales),
                      _ptr(vm), _ptr(K), W, H, ctypes.c_float(0.3), ctypes.c_float(0.01),
                      ctypes.c_float(1e10), ctypes.c_float(0.0), _ptr(radii), _ptr(m2),
                      _ptr(dep), _ptr(con), 0, _stream())
            v2 = torch.randn(1, N, 2, device="cuda", generator=gg)
            vc = torch.randn(1, N, 3, device="cuda", generator=gg) * 1e-3
            vd = torch.randn(1, N, device="cuda", generator=gg)
            vdirs = torch.randn(N, 3, device="cuda", generator=gg)
            vop = torch.randn(N, device="cuda", generator=gg)
            step = opt.step_count + 1
            if fused:
                P = ctypes.c_void_p * 4
                hyper = None
                if dev_factors:
                    fac = adam_factors(lrs, opt.betas, step)
                    hyper = torch.tensor([x for f in fac for x in f], device="cuda")
                _lib.call("gsplat_hip_projection_bwd_adam", N, _ptr(ps[0]), _ptr(ps[2]),
                          _ptr(scales), _ptr(vm), _ptr(K), W, H, ctypes.c_float(0.3),
                          _ptr(radii), _ptr(con), _ptr(v2), _ptr(vd), _ptr(vc), _ptr(vdirs),
                          _ptr(vop), _ptr(opac), P(*[p.data_ptr() for p in ps]),
                          P(*[m.data_ptr() for m in opt.exp_avg]),
                          P(*[v.data_ptr() for v in opt.exp_avg_sq]),
                          (ctypes.c_float * 4)(*lrs), ctypes.c_float(0.9),
                          ctypes.c_float(0.999), ctypes.c_float(1e-15), step, _ptr(hyper), 0,
                          _stream())
                opt.step_count += 1
            else:
                v_means = torch.empty(N, 3, device="cuda")
                v_quats = torch.empty(N, 4, device="cuda")
                v_scales = torch.empty(N, 3, device="cuda")
                _lib.call("gsplat_hip_projection_bwd", 1, N, _ptr(ps[0]), _ptr(ps[2]),
                          _ptr(scales), _ptr(vm), _ptr(K), W, H, ctypes.c_float(0.3),
                          _ptr(radii), _ptr(con), 0, _ptr(v2), _ptr(vd), _ptr(vc), 0,
                          _ptr(v_means), _ptr(v_quats), _ptr(v_scales), 0, _stream())
                opt.params[0].grad, opt.params[2].grad = v_means, v_quats
                opt.step(xform={0: (v_means, vdirs, 1), 1: (v_scales, scales, 2),
                                3: (vop, opac, 3)})
                opt.zero_grad()
            assert (radii > 0).any() and (radii == 0).any()
        torch.cuda.synchronize()
        res.append([p.clone() for p in ps] + [m.clone() for m in opt.exp_avg] +
                   [v.clone() for v in opt.exp_avg_sq])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_trainer_geometry_adam_in_projection_close(monkeypatch):
    """The trainer with the geometry groups' Adam inside the projection
    backward (GSPLAT_HIP_GEOM_IN_PROJ=1, the one-rank default) applies it on
    every step and tracks the trainer that steps FusedAdam after the
    backward (last-bit differences come from the rasterizer's atomics)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    out = {}
    for f in ("0", "1"):
        monkeypatch.setenv("GSPLAT_HIP_GEOM_IN_PROJ", f)
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", max_steps=100)
        assert tr.geom_in_proj == (f == "1")
        losses = []
        for it in range(5):
            losses.append(float(tr.step(it)))
            assert tr.geom_applied == (f == "1")
        out[f] = (losses, {k: p.detach().clone() for k, p in tr.params.items()},
                  [m.clone() for m in tr.opt.exp_avg_sq])
    assert out["0"][0][0] == out["1"][0][0]
    for a, b in zip(out["0"][0], out["1"][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-7, (out["0"][0], out["1"][0])
    for k in out["0"][1]:
        torch.testing.assert_close(out["1"][1][k], out["0"][1][k], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("dev_factors", [False, True])
def test_projection_2dgs_bwd_adam_is_exact(dev_factors):
    """The 2DGS projection backward with the geometry groups' Adam fused in
    (gsplat_hip_projection_2dgs_bwd_adam, ABI 33) updates parameters and
    moments bit for bit as projection_2dgs_bwd + FusedAdam with the trainer's
    gradient transforms (means + v_dirs, exp and sigmoid VJPs), over three
    steps, host and device factor forms, invisible surfels and a ragged N."""
    import ctypes
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    from gsplat_hip.losses import FusedAdam, adam_factors
    g = torch.Generator().manual_seed(4)
    N, W, H = 3001, 320, 240
    means = (torch.randn(N, 3, generator=g) * 0.8 + torch.tensor([0, 0, 4.0])).cuda()
    logs = torch.log(torch.rand(N, 3, generator=g) * 0.05 + 0.005).cuda()
    quats = torch.nn.functional.normalize(torch.randn(N, 4, generator=g), dim=-1).cuda()
    logit = torch.randn(N, generator=g).cuda()
    vm = torch.eye(4)[None].cuda()
    K = torch.tensor([[[300.0, 0, 160], [0, 300.0, 120], [0, 0, 1]]]).cuda()
    lrs = [1.6e-4, 5e-3, 1e-3, 5e-2]
    res = []
    for fused in (False, True):
        ps = [t.clone() for t in (means, logs, quats, logit)]
        opt = FusedAdam([torch.nn.Parameter(p) for p in ps], lrs, betas=(0.9, 0.999), eps=1e-15)
        ps = [p.data for p in opt.params]
        for it in range(3):
            gg = torch.Generator(device="cuda").manual_seed(30 + it)
            scales = torch.exp(ps[1])
            opac = torch.sigmoid(ps[3])
            radii = torch.empty(1, N, dtype=torch.int32, device="cuda")
            m2 = torch.empty(1, N, 2, device="cuda")
            dep = torch.empty(1, N, device="cuda")
            rt = torch.empty(1, N, 3, 3, device="cuda")
            nr = torch.empty(1, N, 3, device="cuda")
            _lib.call("gsplat_hip_projection_2dgs_fwd", 1, N, _ptr(ps[0]), _ptr(ps[2]),
                      _ptr(scales), _ptr(vm), _ptr(K), W, H, ctypes.c_float(0.01),
                      ctypes.c_float(1e10), ctypes.c_float(0.0), _ptr(radii), _ptr(m2),
                      _ptr(dep), _ptr(rt), _ptr(nr), _stream())
            v2 = torch.randn(1, N, 2, device="cuda", generator=gg)
            vrt = torch.randn(1, N, 3, 3, device="cuda", generator=gg) * 1e-3
            vnr = torch.randn(1, N, 3, device="cuda", generator=gg) * 1e-2
            vd = torch.randn(1, N, device="cuda", generator=gg)
            vdirs = torch.randn(N, 3, device="cuda", generator=gg)
            vop = torch.randn(N, device="cuda", generator=gg)
            step = opt.step_count + 1
            if fused:
                P = ctypes.c_void_p * 4
                hyper = None
                if dev_factors:
                    fac = adam_factors(lrs, opt.betas, step)
                    hyper = torch.tensor([x for f in fac for x in f], device="cuda")
                _lib.call("gsplat_hip_projection_2dgs_bwd_adam", N, _ptr(ps[0]), _ptr(ps[2]),
                          _ptr(scales), _ptr(vm), _ptr(K), _ptr(radii), _ptr(rt), _ptr(v2),
                          _ptr(vd), _ptr(vnr), _ptr(vrt), _ptr(vdirs), _ptr(vop), _ptr(opac),
                          P(*[p.data_ptr() for p in ps]),
                          P(*[m.data_ptr() for m in opt.exp_avg]),
                          P(*[v.data_ptr() for v in opt.exp_avg_sq]),
                          (ctypes.c_float * 4)(*lrs), ctypes.c_float(0.9),
                          ctypes.c_float(0.999), ctypes.c_float(1e-15), step, _ptr(hyper), 0,
                          _stream())
                opt.step_count += 1
            else:
                v_means = torch.empty(N, 3, device="cuda")
                v_quats = torch.empty(N, 4, device="cuda")
                v_scales = torch.empty(N, 3, device="cuda")
                _lib.call("gsplat_hip_projection_2dgs_bwd", 1, N, _ptr(ps[0]), _ptr(ps[2]),
                          _ptr(scales), _ptr(vm), _ptr(K), W, H, _ptr(radii), _ptr(rt),
                          _ptr(v2), _ptr(vd), _ptr(vnr), _ptr(vrt), _ptr(v_means),
                          _ptr(v_quats), _ptr(v_scales), 0, _stream())
                opt.params[0].grad, opt.params[2].grad = v_means, v_quats
                opt.step(xform={0: (v_means, vdirs, 1), 1: (v_scales, scales, 2),
                                3: (vop, opac, 3)})
                opt.zero_grad()
            assert (radii > 0).any() and (radii == 0).any()
        torch.cuda.synchronize()
        res.append([p.clone() for p in ps] + [m.clone() for m in opt.exp_avg] +
                   [v.clone() for v in opt.exp_avg_sq])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b), float((a - b).abs().max())


def test_trainer_2dgs_geometry_adam_in_projection_close(monkeypatch):
    """The 2DGS trainer with the geometry Adam inside the surfel projection
    backward (the one-rank default) applies it on every step and tracks the
    trainer that steps FusedAdam after the backward (last-bit differences
    from the rasterizer's atomics)."""
    from gsplat_hip.train_step import Trainer
    means, rgbs, vm, K, W, H = _small_scene()
    out = {}
    for f in ("0", "1"):
        monkeypatch.setenv("GSPLAT_HIP_GEOM_IN_PROJ", f)
        tr = Trainer(means, rgbs, vm, K, W, H, device="cuda", model="2dgs", max_steps=100)
        assert tr.geom_in_proj == (f == "1")
        losses = []
        for it in range(5):
            losses.append(float(tr.step(it)))
            assert tr.geom_applied == (f == "1")
        out[f] = (losses, {k: p.detach().clone() for k, p in tr.params.items()})
    assert out["0"][0][0] == out["1"][0][0]
    for a, b in zip(out["0"][0], out["1"][0]):
        assert abs(a - b) <= 1e-4 * abs(a) + 1e-7, (out["0"][0], out["1"][0])
    for k in out["0"][1]:
        torch.testing.assert_close(out["1"][1][k], out["0"][1][k], rtol=1e-3, atol=1e-5)
