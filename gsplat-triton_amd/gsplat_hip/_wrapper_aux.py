"""Auxiliary ops that the reference's strategies and optimizers call through
its CUDA extension on every backend, backed by
libgsplat_hip.so (csrc/aux_ops.hip):

    quat_scale_to_covar_preci  gsplat/cuda/_wrapper.py:111-142 (autograd :651-689)
    compute_relocation         gsplat/relocation.py:10-51 (MCMCStrategy)
    adam / SelectiveAdam       gsplat/cuda/_wrapper.py:56-69,
                               gsplat/optimizers/selective_adam.py

With these, gsplat.strategy.MCMCStrategy (ops.relocate / sample_add /
inject_noise_to_position) and SelectiveAdam run on the HIP backend.
"""

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._wrapper import _aligned16, _dev_check, _f32c, _ptr, _stream


class _QuatScaleToCovarPreci(torch.autograd.Function):
    """Covariance / precision matrices from quaternions and scales
    (gsplat/cuda/_wrapper.py:651-689)."""

    @staticmethod
    def forward(ctx, quats, scales, compute_covar=True, compute_preci=True, triu=False):
        quats, scales = _aligned16(_f32c(quats)), _f32c(scales)
        _dev_check(quats, scales)
        N = quats.shape[0]
        shape = (N, 6) if triu else (N, 3, 3)
        covars = torch.empty(shape, device=quats.device) if compute_covar else None
        precis = torch.empty(shape, device=quats.device) if compute_preci else None
        _lib.call("gsplat_hip_quat_scale_to_covar_preci_fwd", N, _ptr(quats), _ptr(scales),
                  int(triu), _ptr(covars), _ptr(precis), _stream())
        ctx.save_for_backward(quats, scales)
        ctx.compute_covar, ctx.compute_preci, ctx.triu = compute_covar, compute_preci, triu
        return covars, precis

    @staticmethod
    def backward(ctx, v_covars, v_precis):
        quats, scales = ctx.saved_tensors
        N = quats.shape[0]

        def dense(v):
            if v is None:
                return None
            return _f32c(v.to_dense() if v.is_sparse else v)

        v_covars = dense(v_covars) if ctx.compute_covar else None
        v_precis = dense(v_precis) if ctx.compute_preci else None
        v_quats = torch.empty((N, 4), device=quats.device)
        v_scales = torch.empty((N, 3), device=quats.device)
        _lib.call("gsplat_hip_quat_scale_to_covar_preci_bwd", N, _ptr(quats), _ptr(scales),
                  int(ctx.triu), _ptr(v_covars), _ptr(v_precis), _ptr(v_quats), _ptr(v_scales),
                  _stream())
        return v_quats, v_scales, None, None, None


def quat_scale_to_covar_preci(
    quats: Tensor,  # [N, 4]
    scales: Tensor,  # [N, 3]
    compute_covar: bool = True,
    compute_preci: bool = True,
    triu: bool = False,
) -> Tuple[Optional[Tensor], Optional[Tensor]]:
    """Covariance and precision matrices, [N,3,3] or (triu) [N,6]
    (gsplat/cuda/_wrapper.py:111-142)."""
    assert quats.dim() == 2 and quats.size(1) == 4, quats.size()
    assert scales.dim() == 2 and scales.size(1) == 3, scales.size()
    covars, precis = _QuatScaleToCovarPreci.apply(quats.contiguous(), scales.contiguous(),
                                                  compute_covar, compute_preci, triu)
    return covars if compute_covar else None, precis if compute_preci else None


@torch.no_grad()
def compute_relocation(
    opacities: Tensor,  # [N]
    scales: Tensor,  # [N, 3]
    ratios: Tensor,  # [N]
    binoms: Tensor,  # [n_max, n_max]
) -> Tuple[Tensor, Tensor]:
    """New opacities and scales of relocated Gaussians, MCMC paper Eq. 9
    (gsplat/relocation.py:10-51).  `ratios` is clamped to [1, n_max] in
    place, as the reference does."""
    N = opacities.shape[0]
    n_max, _ = binoms.shape
    assert scales.shape == (N, 3), scales.shape
    assert ratios.shape == (N,), ratios.shape
    ratios.clamp_(min=1, max=n_max)
    opacities, scales, binoms = _f32c(opacities), _f32c(scales), _f32c(binoms)
    r = ratios.int().contiguous()
    _dev_check(opacities, scales, r, binoms)
    new_opacities = torch.empty_like(opacities)
    new_scales = torch.empty_like(scales)
    _lib.call("gsplat_hip_relocation", N, _ptr(opacities), _ptr(scales), _ptr(r), _ptr(binoms),
              int(n_max), _ptr(new_opacities), _ptr(new_scales), _stream())
    return new_opacities, new_scales


@torch.no_grad()
def adam(param: Tensor, param_grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor,
         valid: Optional[Tensor], lr: float, b1: float, b2: float, eps: float) -> None:
    """In-place fused Adam step of the reference (no bias correction) on the
    rows of dim 0 whose `valid` is true (gsplat/cuda/_wrapper.py:56-69,
    AdamCUDA.cu:12-46).  A row is all elements of one Gaussian; the
    reference's kernel indexes `valid` per last-dimension row instead, which
    reads past the mask for [N, K, 3] parameters -- here the mask is per
    Gaussian for every parameter shape."""
    for t in (param, param_grad, exp_avg, exp_avg_sq):
        assert t.is_contiguous() and t.dtype == torch.float32
    _dev_check(param, param_grad, exp_avg, exp_avg_sq, valid)
    n_rows = param.shape[0] if param.dim() > 0 else 1
    row = param.numel() // max(n_rows, 1)
    v = None
    if valid is not None:
        assert valid.numel() == n_rows, (valid.shape, param.shape)
        v = valid.to(torch.uint8).contiguous()
    _lib.call("gsplat_hip_selective_adam", n_rows, row, _ptr(param), _ptr(param_grad),
              _ptr(exp_avg), _ptr(exp_avg_sq), _ptr(v), float(lr), float(b1), float(b2),
              float(eps), _stream())


class SelectiveAdam(torch.optim.Adam):
    """Adam that updates only the visible Gaussians, fused in one launch per
    parameter (gsplat/optimizers/selective_adam.py)."""

    def __init__(self, params, eps, betas):
        super().__init__(params=params, eps=eps, betas=betas)

    @torch.no_grad()
    def step(self, visibility):
        for group in self.param_groups:
            lr, eps = group["lr"], group["eps"]
            beta1, beta2 = group["betas"]
            assert len(group["params"]) == 1, "more than one tensor in group"
            param = group["params"][0]
            if param.grad is None:
                continue
            state = self.state[param]
            if len(state) == 0:
                state["step"] = torch.tensor(0.0, dtype=torch.float32)
                state["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
            adam(param, param.grad, state["exp_avg"], state["exp_avg_sq"], visibility, lr, beta1,
                 beta2, eps)
