"""Fused photometric loss and multi-tensor Adam for the training step.

`l1_ssim_loss` = (1 - lam) * mean|render - gt| + lam * (1 - SSIM_valid),
the loss of examples/simple_trainer.py:642-646 with fused_ssim
(rahul-goel/fused-ssim, padding="valid") restated in HIP (csrc/ssim.hip).
`FusedAdam` applies torch.optim.Adam's update to all Gaussian parameter
groups in one kernel (csrc/adam.hip).
"""

import ctypes
import math
import os

import torch

from . import _lib
from ._wrapper import _ptr, _stream


class _L1SSIM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, img, gt):
        assert img.dim() == 4 and img.shape == gt.shape, (img.shape, gt.shape)
        img = img.contiguous().float()
        gt = gt.contiguous().float()
        B, H, W, C = img.shape
        ws = torch.empty(max(int(_lib.query("gsplat_hip_ssim_workspace_bytes", B, H, W, C)), 4),
                         dtype=torch.uint8, device=img.device)
        sums = torch.empty(2, device=img.device)
        _lib.call("gsplat_hip_ssim_l1_fwd", B, H, W, C, _ptr(img), _ptr(gt), _ptr(sums),
                  _ptr(ws), _stream())
        ctx.save_for_backward(img, gt, ws)
        n_map = B * C * (H - 10) * (W - 10)
        n_img = B * C * H * W
        return sums[0] / n_map, sums[1] / n_img  # mean SSIM, mean L1

    @staticmethod
    def backward(ctx, g_ssim, g_l1):
        img, gt, ws = ctx.saved_tensors
        B, H, W, C = img.shape
        dloss = torch.stack([g_ssim.reshape(()), g_l1.reshape(())]).float().contiguous()
        grad = torch.empty_like(img)
        _lib.call("gsplat_hip_ssim_l1_bwd", B, H, W, C, _ptr(img), _ptr(gt), _ptr(ws),
                  _ptr(dloss), _ptr(grad), _stream())
        return grad, None


def ssim_and_l1(img, gt):
    """(mean SSIM over the valid region, mean L1) of [B,H,W,C] images."""
    return _L1SSIM.apply(img, gt)


class _L1SSIMLoss(torch.autograd.Function):
    """The whole loss in one forward and one backward launch pair: the scalar
    arithmetic is folded into the reduction / gradient kernels."""

    @staticmethod
    def forward(ctx, img, gt, lam):
        assert img.dim() == 4 and img.shape == gt.shape, (img.shape, gt.shape)
        img = img.contiguous().float()
        gt = gt.contiguous().float()
        B, H, W, C = img.shape
        ws = torch.empty(max(int(_lib.query("gsplat_hip_ssim_workspace_bytes", B, H, W, C)), 4),
                         dtype=torch.uint8, device=img.device)
        out = torch.empty(3, device=img.device)
        _lib.call("gsplat_hip_l1_ssim_loss_fwd", B, H, W, C, _ptr(img), _ptr(gt),
                  ctypes.c_float(lam), _ptr(out), _ptr(ws), _stream())
        ctx.save_for_backward(img, gt, ws)
        ctx.lam = float(lam)
        return out[0]

    @staticmethod
    def backward(ctx, g_loss):
        img, gt, ws = ctx.saved_tensors
        B, H, W, C = img.shape
        g_loss = g_loss.float().contiguous()
        grad = torch.empty_like(img)
        _lib.call("gsplat_hip_l1_ssim_loss_bwd", B, H, W, C, _ptr(img), _ptr(gt), _ptr(ws),
                  ctypes.c_float(ctx.lam), _ptr(g_loss), _ptr(grad), _stream())
        return grad, None, None


class _L1SSIMLossFused(torch.autograd.Function):
    """The same loss with dloss/dimg computed in the forward launch
    (csrc/ssim.hip fused_kernel); the backward scales it by the incoming
    gradient.  The training path: no per-pixel SSIM partials through HBM."""

    @staticmethod
    def forward(ctx, img, gt, lam, gt_index=None, out_ring=None, channels=None):
        # gt_index: device int64 [1]; gt is then a stack [n, H, W, C] of
        # single-image targets and gt[gt_index] is this image's target.
        # out_ring: (ring float32 [R], seq int64 [1], both on the device): the
        # loss also goes to ring[(seq - 1) % R] (gsplat_hip_l1_ssim_loss_fused_fwd_ring)
        # channels: the loss reads the first `channels` of img's XS channels
        # (an RGB+D render in place); its gradient is img-shaped, zero in the rest
        XS = img.shape[-1]
        C = XS if channels is None else int(channels)
        if gt_index is None:
            assert img.dim() == 4 and img.shape[:3] == gt.shape[:3] and gt.shape[3] == C, \
                (img.shape, gt.shape)
        else:
            assert img.dim() == 4 and img.shape[0] == 1 and gt.shape[1:3] == img.shape[1:3] \
                and gt.shape[3] == C, (img.shape, gt.shape)
            assert gt_index.dtype == torch.int64 and gt_index.is_cuda and gt.is_contiguous()
        img = img.contiguous().float()
        gt = gt.contiguous().float()
        B, H, W, _ = img.shape
        ws = torch.empty(max(int(_lib.query("gsplat_hip_l1_ssim_loss_fused_workspace_bytes",
                                            B, H, W, C)), 4),
                         dtype=torch.uint8, device=img.device)
        out = torch.empty(3, device=img.device)
        unit = torch.empty_like(img)
        if out_ring is None:
            _lib.call("gsplat_hip_l1_ssim_loss_fused_fwd", B, H, W, C, XS, _ptr(img), _ptr(gt),
                      _ptr(gt_index), ctypes.c_float(lam), _ptr(out), _ptr(unit), _ptr(ws),
                      _stream())
        else:
            ring, seq = out_ring
            assert ring.dtype == torch.float32 and ring.is_cuda and seq.dtype == torch.int64
            _lib.call("gsplat_hip_l1_ssim_loss_fused_fwd_ring", B, H, W, C, XS, _ptr(img), _ptr(gt),
                      _ptr(gt_index), ctypes.c_float(lam), _ptr(out), _ptr(unit), _ptr(ws),
                      _ptr(ring), ring.numel(), _ptr(seq), _stream())
        ctx.save_for_backward(unit)
        return out[0]

    @staticmethod
    def backward(ctx, g_loss):
        (unit,) = ctx.saved_tensors
        if g_loss is ONE_GRAD:  # the trainer's constant 1.0 seed: the unit gradient as is
            return unit, None, None, None, None, None
        g_loss = g_loss.float().contiguous()
        grad = torch.empty_like(unit)
        _lib.call("gsplat_hip_l1_ssim_loss_fused_bwd", unit.numel(), _ptr(unit), _ptr(g_loss),
                  _ptr(grad), _stream())
        return grad, None, None, None, None, None


# A constant scalar 1.0 the trainer seeds loss.backward() with (never written):
# seen as the incoming gradient, the fused loss's backward returns its stored
# unit gradient without the scaling launch.
ONE_GRAD = None

# GSPLAT_HIP_SSIM_FUSED=0: the two-pass loss (partials to HBM) for training too
SSIM_FUSED = os.environ.get("GSPLAT_HIP_SSIM_FUSED", "1") != "0"


def l1_ssim_loss(img, gt, ssim_lambda=0.2, fused=None, gt_index=None, _out_ring=None,
                 _channels=None):
    """(1 - ssim_lambda) * mean L1 + ssim_lambda * (1 - mean SSIM_valid).
    With a gradient to compute (and C in {1, 3}) the one-pass fused kernel
    runs, unless `fused=False` (or GSPLAT_HIP_SSIM_FUSED=0).  `gt_index`
    (device int64 [1], fused kernel only): `gt` is a stack of targets and
    gt[gt_index] the one of this [1, H, W, C] image -- chosen on the device,
    no copy (the captured training step).  `_out_ring` (internal, with
    gt_index): (ring, seq) device tensors; the loss value is also written to
    ring[(seq - 1) % len(ring)] by the reduction launch (graph_step.py).
    `_channels` (internal): the loss is over img[..., :_channels] (an RGB+D
    render read in place by the fused kernel; its gradient is img-shaped)."""
    if _channels is not None and _channels != img.shape[-1]:
        if fused is None:
            fused = SSIM_FUSED and torch.is_grad_enabled() and img.requires_grad
        if not (fused and img.dim() == 4 and _channels in (1, 3)):
            img = img[..., :_channels]  # the generic path on the slice
        else:
            return _L1SSIMLossFused.apply(img, gt, float(ssim_lambda), gt_index, _out_ring,
                                          int(_channels))
    if fused is None:
        fused = SSIM_FUSED and torch.is_grad_enabled() and img.requires_grad
    if gt_index is not None:
        if not (fused and img.dim() == 4 and img.shape[-1] in (1, 3)):
            raise ValueError("l1_ssim_loss: gt_index needs the fused kernel (grad, C in {1, 3})")
        return _L1SSIMLossFused.apply(img, gt, float(ssim_lambda), gt_index, _out_ring)
    if fused and img.dim() == 4 and img.shape[-1] in (1, 3):
        return _L1SSIMLossFused.apply(img, gt, float(ssim_lambda))
    return _L1SSIMLoss.apply(img, gt, float(ssim_lambda))


def adam_factors(lrs, betas, step):
    """The per-group factors gsplat_hip_adam_step computes on the host, with
    its arithmetic (float lr and beta promoted to double, double pow / sqrt,
    rounded to float): [lr_i / (1 - beta1^t), 1 / sqrt(1 - beta2^t)] per
    group -- what the captured step's device-side variants read."""
    import numpy as np
    b1, b2 = float(np.float32(betas[0])), float(np.float32(betas[1]))
    bc1, bc2 = 1.0 - b1 ** int(step), 1.0 - b2 ** int(step)
    ib = float(np.float32(1.0 / math.sqrt(bc2)))
    return [(float(np.float32(float(np.float32(lr)) / bc1)), ib) for lr in lrs]


def adam_groups(params, grads, exp_avgs, exp_avg_sqs, lrs, betas, eps, step, aux=None,
                modes=None, hyper=None, skip=None):
    """One fused Adam launch (csrc/adam.hip) over flat float32 tensors: group
    i updates params[i] in place from grads[i] (None = zero) with its lr.
    aux/modes form the gradient in-register (gsplat_hip_adam_step_ex); hyper (device
    f32[2 n], adam_factors' values) / skip (device i32 flag): the captured
    step's form (gsplat_hip_adam_step_dev; lrs and step unused)."""
    n = len(params)
    P = ctypes.c_void_p * n
    for t in list(params) + list(exp_avgs) + list(exp_avg_sqs):
        assert t.is_contiguous() and t.dtype == torch.float32
    head = [n, P(*[p.data_ptr() for p in params]),
            P(*[0 if g is None else g.data_ptr() for g in grads])]
    if hyper is not None:
        assert hyper.dtype == torch.float32 and hyper.numel() >= 2 * n
        ax = [None] * n if aux is None else aux
        for a in ax:
            assert a is None or (a.is_contiguous() and a.dtype == torch.float32)
        _lib.call("gsplat_hip_adam_step_dev", *head,
                  P(*[0 if a is None else a.data_ptr() for a in ax]),
                  (ctypes.c_int32 * n)(*[int(m) for m in (modes or [0] * n)]),
                  P(*[m.data_ptr() for m in exp_avgs]), P(*[v.data_ptr() for v in exp_avg_sqs]),
                  (ctypes.c_int64 * n)(*[p.numel() for p in params]), hyper.data_ptr(),
                  float(betas[0]), float(betas[1]), float(eps),
                  0 if skip is None else skip.data_ptr(), _stream())
        return
    tail = [P(*[m.data_ptr() for m in exp_avgs]), P(*[v.data_ptr() for v in exp_avg_sqs]),
            (ctypes.c_int64 * n)(*[p.numel() for p in params]),
            (ctypes.c_float * n)(*[float(x) for x in lrs]), float(betas[0]), float(betas[1]),
            float(eps), int(step)]
    if modes is not None and any(modes):
        for a in aux:
            assert a is None or (a.is_contiguous() and a.dtype == torch.float32)
        _lib.call("gsplat_hip_adam_step_ex", *head,
                  P(*[0 if a is None else a.data_ptr() for a in aux]),
                  (ctypes.c_int32 * n)(*[int(m) for m in modes]), *tail, _stream())
        return
    _lib.call("gsplat_hip_adam_step", *(head + tail), _stream())


class FusedAdam:
    """torch.optim.Adam semantics (per-group lr, shared betas/eps) in one launch.

    (A variant that deferred the SH groups' update to a side stream, to
    overlap the next step's projection and isect, measured slower at M2 --
    620-650 against 660 images/s, profiles/r2_s4_defer: the two split the HBM
    bandwidth instead of filling each other's gaps -- and was removed.)"""

    def __init__(self, params, lrs, betas=(0.9, 0.999), eps=1e-8):
        self.params = list(params)
        self.lrs = [float(x) for x in lrs]
        self.betas, self.eps = betas, eps
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in self.params]
        self.step_count = 0
        for p in self.params:
            assert p.is_contiguous() and p.dtype == torch.float32

    def _launch(self, idx, grads, xform=None, hyper=None, void=None):
        aux = modes = None
        if xform:
            aux = [xform[i][1] if i in xform else None for i in idx]
            modes = [xform[i][2] if i in xform else 0 for i in idx]
            grads = [xform[i][0] if i in xform else g for i, g in enumerate(grads)]
        adam_groups([self.params[i].data for i in idx], [grads[i] for i in idx],
                    [self.exp_avg[i] for i in idx], [self.exp_avg_sq[i] for i in idx],
                    [self.lrs[i] for i in idx], self.betas, self.eps, self.step_count,
                    aux, modes, hyper, void)

    @torch.no_grad()
    def step(self, skip=(), xform=None, hyper=None, void=None):
        """skip: indices already updated for this step (by the SH backward
        with the update fused in, train_step.Trainer).  xform: {index:
        (grad, aux, mode)} -- the gradient of that group formed in-register
        (adam_step_ex modes: 1 sum, 2 exp VJP, 3 sigmoid VJP).  hyper / void:
        the captured step's device-side factors of the launched groups (in
        launch order, adam_factors) and void-step flag (step_count is then
        the caller's business)."""
        if hyper is None:
            self.step_count += 1
        grads = [p.grad for p in self.params]
        for gr in grads:
            assert gr is None or gr.is_contiguous()
        idx = [i for i in range(len(self.params)) if i not in skip]
        if idx:
            self._launch(idx, grads, xform=xform, hyper=hyper, void=void)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None
