"""DefaultStrategy's densification on the HIP backend (csrc/strategy.hip).

`DefaultStrategyConfig` carries the reference's DefaultStrategy fields and
defaults (gsplat/strategy/default.py:79-95) and its schedule
(`step_post_backward`, default.py:175-211).  `refine` is _grow_gs + _prune_gs
(default.py:264-340) over duplicate / split / remove (ops.py:86-211) as one
compaction of every parameter and both Adam moments: a plan launch, the one
host read of the four totals, and an apply launch that writes each array's
final layout once.  `reset_opacity` is reset_opa (ops.py:214-243).

The reference's optimizer-state surgery (moments of new rows start at zero,
removed rows drop theirs, the step counter is kept) is applied to whatever
moment tensors the caller passes; the trainer passes its fused Adam's state.
"""

import ctypes
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._wrapper import _ptr, _stream

COPY, MEANS, SCALES, OPACITIES, MOMENT = 0, 1, 2, 3, 4
_KIND = {"means": MEANS, "scales": SCALES, "opacities": OPACITIES}


@dataclass
class DefaultStrategyConfig:
    """Fields and defaults of gsplat.strategy.DefaultStrategy (default.py:79-95)."""
    prune_opa: float = 0.005
    grow_grad2d: float = 0.0002
    grow_scale3d: float = 0.01
    grow_scale2d: float = 0.05
    prune_scale3d: float = 0.1
    prune_scale2d: float = 0.15
    refine_scale2d_stop_iter: int = 0
    refine_start_iter: int = 500
    refine_stop_iter: int = 15_000
    reset_every: int = 3000
    refine_every: int = 100
    pause_refine_after_reset: int = 0
    absgrad: bool = False
    revised_opacity: bool = False
    key_for_gradient: str = "means2d"

    def is_refine_step(self, step: int) -> bool:
        """default.py:175-183 (with the refine_stop_iter early return)."""
        return (self.refine_start_iter < step < self.refine_stop_iter
                and step % self.refine_every == 0
                and step % self.reset_every >= self.pause_refine_after_reset)

    def is_reset_step(self, step: int) -> bool:
        """default.py:205-211."""
        return step < self.refine_stop_iter and step % self.reset_every == 0


def _check(t: Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"densify: {name} must be on the GPU")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise ValueError(f"densify: {name} must be contiguous float32")


@torch.no_grad()
def refine(params: Dict[str, Tensor], moments: Dict[str, List[Tensor]], grad2d: Tensor,
           count: Tensor, step: int, cfg: DefaultStrategyConfig, scene_scale: float = 1.0,
           generator: Optional[torch.Generator] = None, z: Optional[Tensor] = None,
           radii2d: Optional[Tensor] = None
           ) -> Tuple[Dict[str, Tensor], Dict[str, List[Tensor]], Tuple[int, int, int]]:
    """Grow + prune (one refine step).  `params`: name -> [N, ...] float32
    (means [N,3], scales [N,3] log, quats [N,4], opacities [N] logits, any
    others copied); `moments`: name -> list of optimizer-state tensors shaped
    like the parameter.  The split noise is z if given, else
    randn(2, n_split, 3) from `generator` on the device.  Returns the new
    parameter and moment tensors and (n_dupli, n_split, n_prune)."""
    for k in ("means", "scales", "quats", "opacities"):
        assert k in params, f"{k} is required in params but missing."
    means, log_scales = params["means"], params["scales"]
    quats, logits = params["quats"], params["opacities"]
    N = means.shape[0]
    dev = means.device
    for k, t in params.items():
        _check(t, k)
        assert t.shape[0] == N, (k, t.shape)
    for k, ms in moments.items():
        for t in ms:
            _check(t, f"moment of {k}")
            assert t.shape == params[k].shape, (k, t.shape)
    assert means.shape == (N, 3) and log_scales.shape == (N, 3) and quats.shape == (N, 4)
    assert logits.numel() == N
    grad2d = grad2d.contiguous().float()
    count = count.contiguous().float()
    assert grad2d.numel() == N and count.numel() == N
    if radii2d is not None:
        radii2d = radii2d.contiguous().float()
    ws = torch.empty(max(int(_lib.query("gsplat_hip_densify_workspace_bytes", N)), 8),
                     dtype=torch.uint8, device=dev)
    totals = torch.empty(5, dtype=torch.int64, device=dev)
    st = _stream()
    _lib.call("gsplat_hip_densify_plan", N, _ptr(grad2d), _ptr(count), _ptr(log_scales),
              _ptr(logits), _ptr(radii2d), ctypes.c_float(cfg.grow_grad2d),
              ctypes.c_float(cfg.grow_scale3d * scene_scale), ctypes.c_float(cfg.prune_opa),
              int(step > cfg.reset_every), ctypes.c_float(cfg.prune_scale3d * scene_scale),
              ctypes.c_float(cfg.grow_scale2d), ctypes.c_float(cfg.prune_scale2d),
              int(cfg.revised_opacity), _ptr(ws), _ptr(totals), st)
    # the one host sync of a refine step
    n_keep, n_dup_kept, n_child_kept, n_split, n_dupli = (int(x) for x in totals.tolist())
    n_out = n_keep + n_dup_kept + 2 * n_child_kept
    if z is None:
        z = torch.randn(2, n_split, 3, device=dev, generator=generator)
    z = z.to(device=dev, dtype=torch.float32).contiguous()
    assert z.shape == (2, n_split, 3), (z.shape, n_split)

    srcs, dsts, rows, kinds = [], [], [], []
    new_params, new_moments = {}, {}
    for k, t in params.items():
        out = torch.empty((n_out,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        new_params[k] = out
        srcs.append(t)
        dsts.append(out)
        rows.append(math.prod(t.shape[1:]))
        kinds.append(_KIND.get(k, COPY))
    for k, ms in moments.items():
        new_moments[k] = []
        for t in ms:
            out = torch.empty((n_out,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            new_moments[k].append(out)
            srcs.append(t)
            dsts.append(out)
            rows.append(math.prod(t.shape[1:]))
            kinds.append(MOMENT)
    n = len(srcs)
    P = ctypes.c_void_p * n
    _lib.call("gsplat_hip_densify_apply", N, _ptr(ws), _ptr(totals), _ptr(z),
              int(cfg.revised_opacity), n, P(*[s.data_ptr() for s in srcs]),
              P(*[d.data_ptr() for d in dsts]), (ctypes.c_int32 * n)(*rows),
              (ctypes.c_int32 * n)(*kinds), _ptr(means), _ptr(quats), _ptr(log_scales),
              _ptr(logits), st)
    # the reference's counts (default.py:185-197): duplicated, split, and
    # pruned among the N + n_dupli + n_split Gaussians after growing
    return new_params, new_moments, (n_dupli, n_split, N + n_dupli + n_split - n_out)


@torch.no_grad()
def reset_opacity(params: Dict[str, Tensor], moments: Dict[str, List[Tensor]], value: float):
    """reset_opa (ops.py:214-243) in place: opacity logits clamped to
    logit(value) (computed in float32 as the reference's
    torch.logit(torch.tensor(value))), their moments zeroed."""
    lim = float(torch.logit(torch.tensor(value, dtype=torch.float32)))
    params["opacities"].clamp_(max=lim)
    for t in moments.get("opacities", []):
        t.zero_()


__all__ = ["DefaultStrategyConfig", "refine", "reset_opacity"]
