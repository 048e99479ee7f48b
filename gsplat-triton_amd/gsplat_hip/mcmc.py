"""MCMCStrategy on the HIP backend (gsplat/strategy/mcmc.py, ops.py:244-369).

`MCMCStrategyConfig` carries the reference's MCMCStrategy fields and defaults
(mcmc.py:49-55) and its schedule (step_post_backward, mcmc.py:103-145):
every `refine_every` steps inside (refine_start_iter, refine_stop_iter) the
dead Gaussians (opacity <= min_opacity) are relocated onto live ones sampled
by opacity (`relocate`, ops.py:244-297) and 5 % new ones are sampled in
(`sample_add`, ops.py:300-340, up to cap_max); every step the positions get
noise shaped by each Gaussian's covariance (`inject_noise`, ops.py:343-369).

The relocated / added Gaussians' opacities and scales come from the
relocation kernel (MCMC paper Eq. 9, csrc/aux_ops.hip); the noise is one
fused launch (gsplat_hip_mcmc_inject_noise) on torch's normal draw, so a
seeded generator gives the reference's sequence of draws.  The optimizer
state follows the reference's surgery (_update_param_with_optimizer):
relocate zeroes the moments of the sampled rows (the dead rows keep
theirs), sample_add appends zero moments.
"""

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._wrapper import _aligned16, _ptr, _stream
from ._wrapper_aux import compute_relocation

N_MAX = 51  # mcmc.py:57-64: binomial table size


@dataclass
class MCMCStrategyConfig:
    """Fields and defaults of gsplat.strategy.MCMCStrategy (mcmc.py:49-55)."""
    cap_max: int = 1_000_000
    noise_lr: float = 5e5
    refine_start_iter: int = 500
    refine_stop_iter: int = 25_000
    refine_every: int = 100
    min_opacity: float = 0.005
    verbose: bool = False

    def is_refine_step(self, step: int) -> bool:
        """mcmc.py:122-126."""
        return (self.refine_start_iter < step < self.refine_stop_iter
                and step % self.refine_every == 0)


def binoms(device=None, n_max: int = N_MAX) -> Tensor:
    """initialize_state's table binoms[n, k] = C(n, k) (mcmc.py:57-64)."""
    t = torch.zeros((n_max, n_max))
    for n in range(n_max):
        for k in range(n + 1):
            t[n, k] = math.comb(n, k)
    return t.to(device) if device is not None else t


def multinomial_sample(weights: Tensor, n: int,
                       generator: Optional[torch.Generator] = None) -> Tensor:
    """n draws with replacement, P(i) proportional to weights[i]
    (_multinomial_sample, ops.py:14-44).  torch.multinomial up to its 2^24
    category limit; above it the reference samples on the host with numpy,
    here by inverse CDF on the device (a cumulative sum and a binary search
    of n uniforms)."""
    if weights.numel() <= 2 ** 24:
        return torch.multinomial(weights, n, replacement=True, generator=generator)
    cdf = torch.cumsum(weights.double(), 0)
    u = torch.rand(n, device=weights.device, dtype=torch.float64, generator=generator) * cdf[-1]
    return torch.searchsorted(cdf, u, right=True).clamp_(max=weights.numel() - 1)


def _relocation(params: Dict[str, Tensor], sampled: Tensor, binoms_t: Tensor,
                min_opacity: float) -> Tuple[Tensor, Tensor]:
    """New opacity logits and log-scales of the sampled rows (ops.py:267-278,
    309-320): Eq. 9 with ratio = 1 + the times each row was drawn."""
    opac = torch.sigmoid(params["opacities"]).flatten()
    eps = torch.finfo(torch.float32).eps
    new_o, new_s = compute_relocation(
        opacities=opac[sampled], scales=torch.exp(params["scales"])[sampled],
        ratios=torch.bincount(sampled)[sampled] + 1, binoms=binoms_t)
    new_o = torch.clamp(new_o, max=1.0 - eps, min=min_opacity)
    return torch.logit(new_o), torch.log(new_s)


@torch.no_grad()
def relocate(params: Dict[str, Tensor], moments: Dict[str, List[Tensor]], dead: Tensor,
             binoms_t: Tensor, min_opacity: float = 0.005,
             generator: Optional[torch.Generator] = None,
             sampled: Optional[Tensor] = None) -> int:
    """relocate (ops.py:244-297) in place: each dead row takes a copy of a
    live row drawn by opacity, and the drawn rows' opacity / scale are
    re-derived so the pair renders as the one did.  Returns the dead count
    (the one host sync).  `sampled`: the draws as indices into the live rows
    (tests: the reference's recorded draws), else drawn from `generator`."""
    dead_idx = dead.nonzero(as_tuple=True)[0]
    n = int(dead_idx.numel())
    if n == 0:
        return 0
    alive_idx = (~dead).nonzero(as_tuple=True)[0]
    if sampled is None:
        probs = torch.sigmoid(params["opacities"]).flatten()[alive_idx]
        sampled = multinomial_sample(probs, n, generator)
    assert sampled.numel() == n, (sampled.shape, n)
    sampled = alive_idx[sampled.to(alive_idx.device)]
    logit, log_s = _relocation(params, sampled, binoms_t, min_opacity)
    params["opacities"][sampled] = logit.reshape((-1,) + params["opacities"].shape[1:])
    params["scales"][sampled] = log_s
    for t in params.values():
        t[dead_idx] = t[sampled]
    for ms in moments.values():
        for v in ms:
            v[sampled] = 0
    return n


@torch.no_grad()
def sample_add(params: Dict[str, Tensor], moments: Dict[str, List[Tensor]], n: int,
               binoms_t: Tensor, min_opacity: float = 0.005,
               generator: Optional[torch.Generator] = None, sampled: Optional[Tensor] = None
               ) -> Tuple[Dict[str, Tensor], Dict[str, List[Tensor]]]:
    """sample_add (ops.py:300-340): n rows drawn by opacity are re-derived
    (as relocate's) and appended as copies; their moments start at zero.
    Returns the new parameter and moment tensors (the inputs' drawn rows are
    updated in place, as the reference's).  `sampled`: given draws (tests)."""
    if sampled is None:
        probs = torch.sigmoid(params["opacities"]).flatten()
        sampled = multinomial_sample(probs, n, generator)
    sampled = sampled.to(params["means"].device)
    assert sampled.numel() == n, (sampled.shape, n)
    logit, log_s = _relocation(params, sampled, binoms_t, min_opacity)
    params["opacities"][sampled] = logit.reshape((-1,) + params["opacities"].shape[1:])
    params["scales"][sampled] = log_s
    new_p = {k: torch.cat([t, t[sampled]]) for k, t in params.items()}
    new_m = {k: [torch.cat([v, v.new_zeros((n,) + tuple(v.shape[1:]))]) for v in ms]
             for k, ms in moments.items()}
    return new_p, new_m


@torch.no_grad()
def inject_noise(params: Dict[str, Tensor], scaler: float,
                 generator: Optional[torch.Generator] = None,
                 z: Optional[Tensor] = None, seed: Optional[int] = None, step: int = 0,
                 step_dev: Optional[Tensor] = None, scaler_dev: Optional[Tensor] = None,
                 skip: Optional[Tensor] = None) -> None:
    """inject_noise_to_position (ops.py:343-369) in place: means +=
    Sigma (z * op_sigmoid(1 - opacity) * scaler), one fused HIP launch.
    The draw z ~ N(0, 1) [N, 3]: `z` if given; else with a `seed`, made in
    the kernel (Philox-4x32-10 keyed by the seed, counter (gaussian, step): a
    pure function of (seed, step, gaussian) -- the trainer's draw, identical
    when a captured step is replayed or re-run); else torch's
    randn_like(means) from `generator` (the reference's draw).  step_dev /
    scaler_dev (int64 [1] / float32 [1] on the device) override step /
    scaler, skip (int32 [1]) voids the launch when non-zero: the captured
    training step's inputs."""
    means = params["means"]
    if not means.is_cuda:
        raise ValueError("mcmc.inject_noise: tensors must be on the GPU")
    N = means.shape[0]
    for k, t in params.items():
        if k in ("means", "quats", "scales", "opacities"):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"mcmc.inject_noise: {k} must be contiguous float32")
    assert means.shape == (N, 3) and params["scales"].shape == (N, 3)
    assert params["quats"].shape == (N, 4) and params["opacities"].numel() == N
    if z is None and seed is None:
        z = torch.randn(means.shape, device=means.device, generator=generator)
    if z is not None:
        z = z.to(device=means.device, dtype=torch.float32).contiguous()
        assert z.shape == (N, 3), z.shape
    for t, dt in ((step_dev, torch.int64), (scaler_dev, torch.float32), (skip, torch.int32)):
        assert t is None or (t.is_cuda and t.dtype == dt and t.numel() >= 1), (t, dt)
    quats = _aligned16(params["quats"])
    _lib.call("gsplat_hip_mcmc_inject_noise", N, _ptr(means), _ptr(quats),
              _ptr(params["scales"]), _ptr(params["opacities"]), _ptr(z),
              int(seed or 0) & 0xFFFFFFFFFFFFFFFF, int(step), _ptr(step_dev), float(scaler),
              _ptr(scaler_dev), _ptr(skip), _stream())


@torch.no_grad()
def inject_noise_to_position(params, optimizers, state, scaler: float) -> None:
    """Drop-in for gsplat.strategy.ops.inject_noise_to_position (ops.py:343-369),
    same signature and draw (torch.randn_like(params["means"]) from the
    global generator), one fused launch instead of the covariance launch and
    the torch passes around it (`ops.inject_noise_to_position =
    gsplat_hip.mcmc.inject_noise_to_position` under the reference's
    MCMCStrategy).  `optimizers` / `state` are unused, as in the reference."""
    z = torch.randn_like(params["means"])
    inject_noise({k: params[k].data for k in ("means", "quats", "scales", "opacities")},
                 scaler, z=z)


def n_to_add(n: int, cap_max: int) -> int:
    """_add_new_gs's count (mcmc.py:175-177)."""
    return max(0, min(cap_max, int(1.05 * n)) - n)


__all__ = ["MCMCStrategyConfig", "binoms", "multinomial_sample", "relocate", "sample_add",
           "inject_noise", "inject_noise_to_position", "n_to_add"]
