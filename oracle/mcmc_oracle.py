"""CPU oracle for MCMCStrategy's refine and position noise -- TEST
INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

numpy restatement of the reference's torch code
(hieu1999210/gsplat-triton @ /root/reference), with the random draws given:
  relocate       gsplat/strategy/ops.py:244-297
  sample_add     gsplat/strategy/ops.py:300-340
  inject_noise   gsplat/strategy/ops.py:343-369
  step           gsplat/strategy/mcmc.py:103-187 (schedule + the two refines)
Pinned to the reference itself: tests/golden/make_golden_mcmc.py runs the
reference's MCMCStrategy.step_post_backward (recording its draws) into
tests/golden/mcmc_*.npz, which tests/test_mcmc.py checks this file against.
"""

import numpy as np

from . import aux_oracle as A

f32 = np.float32


def _sigmoid(x):
    return (1.0 / (1.0 + np.exp(-np.asarray(x, np.float64)))).astype(f32)


def _relocated(params, sampled, binoms, min_opacity):
    """ops.py:267-278: Eq. 9 on the drawn rows, ratio = 1 + times drawn."""
    o = _sigmoid(params["opacities"]).reshape(-1)
    ratios = np.bincount(sampled)[sampled] + 1
    ratios = np.clip(ratios, 1, binoms.shape[0])
    no, ns = A.relocation(o[sampled], np.exp(params["scales"][sampled]), ratios, binoms)
    eps = np.finfo(np.float32).eps
    no = np.clip(no, min_opacity, 1.0 - eps).astype(f32)
    return np.log(no / (1.0 - no)).astype(f32), np.log(ns).astype(f32)


def relocate(params, moments, dead, sampled_alive, binoms, min_opacity=0.005):
    """In place on copies: returns (params, moments)."""
    params = {k: v.copy() for k, v in params.items()}
    moments = {k: [v.copy() for v in ms] for k, ms in moments.items()}
    dead_idx = np.nonzero(dead)[0]
    if dead_idx.size == 0:
        return params, moments
    alive_idx = np.nonzero(~dead)[0]
    sampled = alive_idx[sampled_alive]
    logit, log_s = _relocated(params, sampled, binoms, min_opacity)
    params["opacities"][sampled] = logit.reshape((-1,) + params["opacities"].shape[1:])
    params["scales"][sampled] = log_s
    for v in params.values():
        v[dead_idx] = v[sampled]
    for ms in moments.values():
        for v in ms:
            v[sampled] = 0
    return params, moments


def sample_add(params, moments, sampled, binoms, min_opacity=0.005):
    params = {k: v.copy() for k, v in params.items()}
    logit, log_s = _relocated(params, sampled, binoms, min_opacity)
    params["opacities"][sampled] = logit.reshape((-1,) + params["opacities"].shape[1:])
    params["scales"][sampled] = log_s
    new_p = {k: np.concatenate([v, v[sampled]]) for k, v in params.items()}
    new_m = {k: [np.concatenate([v, np.zeros((len(sampled),) + v.shape[1:], f32)]) for v in ms]
             for k, ms in moments.items()}
    return new_p, new_m


def inject_noise(params, z, scaler):
    """means + Sigma (z * op_sigmoid(1 - o) * scaler), op_sigmoid k=100, x0=0.995."""
    params = dict(params)
    o = _sigmoid(params["opacities"]).reshape(-1).astype(np.float64)
    f = 1.0 / (1.0 + np.exp(-100.0 * ((1.0 - o) - 0.995)))
    cov, _ = A.covar_preci(params["quats"], np.exp(params["scales"]))
    w = np.asarray(z, np.float64) * (f * scaler)[:, None]
    params["means"] = (params["means"] + np.einsum("bij,bj->bi", cov.astype(np.float64), w)
                       ).astype(f32)
    return params


def binoms(n_max=51):
    from math import comb
    b = np.zeros((n_max, n_max), f32)
    for n in range(n_max):
        for k in range(n + 1):
            b[n, k] = comb(n, k)
    return b


def step(params, moments, step_i, lr, z, reloc_idx, add_idx, cap_max=1_000_000,
         noise_lr=5e5, min_opacity=0.005, refine_start_iter=500, refine_stop_iter=25_000,
         refine_every=100):
    """MCMCStrategy.step_post_backward (mcmc.py:103-145) with the draws given."""
    b = binoms()
    if refine_start_iter < step_i < refine_stop_iter and step_i % refine_every == 0:
        dead = _sigmoid(params["opacities"]).reshape(-1) <= min_opacity
        params, moments = relocate(params, moments, dead, reloc_idx, b, min_opacity)
        n = params["means"].shape[0]
        n_add = max(0, min(cap_max, int(1.05 * n)) - n)
        if n_add > 0:
            params, moments = sample_add(params, moments, add_idx, b, min_opacity)
    params = inject_noise(params, z, lr * noise_lr)
    return params, moments
