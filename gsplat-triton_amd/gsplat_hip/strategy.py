"""Trainer glue of the training step as single HIP launches (csrc/strategy.hip).

`activate`     -- exp(log_scales), sigmoid(logits) with autograd, the
                  activations of examples/simple_trainer.py:565-566.
`update_state_` -- DefaultStrategy._update_state for packed=False
                  (gsplat/strategy/default.py:213-262), in place, no host sync.
"""

import ctypes

import torch

from . import _lib
from ._wrapper import _f32c, _ptr, _stream


def _dev(*ts):
    for t in ts:
        if not t.is_cuda:
            raise ValueError("gsplat_hip.strategy: tensors must be on the GPU")


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_scales, logits, fusion=None, fetch=None):
        log_scales, logits = _f32c(log_scales), _f32c(logits)
        _dev(log_scales, logits)
        scales = torch.empty_like(log_scales)
        opac = torch.empty_like(logits)
        if fetch is not None:  # the captured step's input block, same launch
            ring, slot_bytes, n_ring, seq, blk = fetch
            _lib.call("gsplat_hip_activate_fwd_fetch", log_scales.numel(), logits.numel(),
                      _ptr(log_scales), _ptr(logits), _ptr(scales), _ptr(opac), ring,
                      int(slot_bytes), int(n_ring), _ptr(seq), _ptr(blk), _stream())
        else:
            _lib.call("gsplat_hip_activate_fwd", log_scales.numel(), logits.numel(),
                      _ptr(log_scales), _ptr(logits), _ptr(scales), _ptr(opac), _stream())
        ctx.save_for_backward(scales, opac)
        # an output without a gradient arrives as None, not as a zero-filled
        # tensor (the geometry Adam in the projection backward leaves scales'
        # gradient None: a [N, 3] fill launch per step otherwise)
        ctx.set_materialize_grads(False)
        ctx.fusion = fusion
        if fusion is not None and fusion.geom_adam is not None:
            fusion.opac_act = opac  # sigmoid(logits), for the geometry Adam's VJP
        return scales, opac

    @staticmethod
    def backward(ctx, v_scales, v_opac):
        scales, opac = ctx.saved_tensors
        if ctx.fusion is not None and ctx.fusion.geom_adam is not None \
                and ctx.fusion.geom_adam.applied and not ctx.fusion.act_taken:
            # the projection backward already ran the geometry Adam with these
            # gradients (v_scales never left it; v_opac came through the tap)
            ctx.fusion.act_taken = True
            return None, None, None, None
        # the trainer's geometry update applies the VJPs in-register
        # (adam_step_ex modes 2 / 3): hand over the incoming gradients
        if ctx.fusion is not None and ctx.fusion.take_activation_grads(
                None if v_scales is None else _f32c(v_scales),
                None if v_opac is None else _f32c(v_opac), scales, opac):
            return None, None, None, None
        v_scales = torch.zeros_like(scales) if v_scales is None else _f32c(v_scales)
        v_opac = torch.zeros_like(opac) if v_opac is None else _f32c(v_opac)
        v_log = torch.empty_like(scales)
        v_logit = torch.empty_like(opac)
        _lib.call("gsplat_hip_activate_bwd", scales.numel(), opac.numel(), _ptr(scales),
                  _ptr(opac), _ptr(v_scales), _ptr(v_opac), _ptr(v_log), _ptr(v_logit),
                  _stream())
        return v_log, v_logit, None, None


def activate(log_scales, logits, fusion=None, fetch=None):
    """(exp(log_scales), sigmoid(logits)), differentiable.  `fusion`: a
    training step's _wrapper.StepFusion whose geometry update takes the
    incoming gradients instead (the VJPs are then formed inside Adam).
    `fetch` = (ring device pointer, slot bytes, slots, seq, block): the same
    launch also performs gsplat_hip_step_fetch (graph_step.GraphStep)."""
    return _Activate.apply(log_scales, logits, fusion, fetch)


@torch.no_grad()
def update_state_(grad2d, count, means2d_grad, radii, width, height, n_cameras, skip=None):
    """grad2d/count += DefaultStrategy's per-step statistics (in place).
    skip: device i32 flag; non-zero leaves the statistics alone (a void
    step of a captured training step)."""
    C, N = radii.shape
    g = _f32c(means2d_grad)
    radii = radii.to(torch.int32).contiguous()
    _dev(grad2d, count, g, radii)
    assert grad2d.is_contiguous() and count.is_contiguous() and grad2d.numel() == N
    _lib.call("gsplat_hip_update_state", C, N, _ptr(g), _ptr(radii),
              ctypes.c_float(width / 2.0 * n_cameras), ctypes.c_float(height / 2.0 * n_cameras),
              _ptr(grad2d), _ptr(count), _ptr(skip), _stream())
