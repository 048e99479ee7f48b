"""Golden vectors for MCMCStrategy.step_post_backward from the REFERENCE's own
torch code (gsplat/strategy/mcmc.py:103-187 over ops.py:244-369: relocate,
sample_add, inject_noise_to_position) with real `torch.optim.Adam`
optimizers, run on the CPU.  Run in the build container only:

    python tests/golden/make_golden_mcmc.py

Harness-only shims (nothing under /root/reference is modified or copied):
the `gsplat` package root is a stub (its __init__ pulls in the CUDA
extension); `quat_scale_to_covar_preci` is the reference's own torch
implementation (gsplat/cuda/_torch_impl.py:41-68) and `compute_relocation`
the oracle's restatement of RelocationCUDA.cu (oracle/aux_oracle.py, the
reference wrapper's in-place clamp kept).  `_multinomial_sample` and
`torch.randn_like` are wrapped to RECORD the draws (the reference's own
calls run), so the HIP path can be fed the identical indices and noise.
Only arrays are committed.
"""

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
NAMES = ("means", "scales", "quats", "opacities", "sh0", "shN")


def _import_reference():
    sys.path.insert(0, ROOT)
    from oracle import aux_oracle as A
    pkg = types.ModuleType("gsplat")
    pkg.__path__ = [os.path.join(REF, "gsplat")]
    sys.modules["gsplat"] = pkg
    from gsplat.cuda._torch_impl import _quat_scale_to_covar_preci
    pkg.quat_scale_to_covar_preci = _quat_scale_to_covar_preci

    def compute_relocation(opacities, scales, ratios, binoms):
        n_max = binoms.shape[0]
        ratios.clamp_(min=1, max=n_max)  # gsplat/relocation.py:43
        no, ns = A.relocation(opacities.numpy(), scales.numpy(), ratios.int().numpy(),
                              binoms.numpy())
        return torch.from_numpy(no), torch.from_numpy(ns)

    reloc = types.ModuleType("gsplat.relocation")
    reloc.compute_relocation = compute_relocation
    sys.modules["gsplat.relocation"] = reloc
    from gsplat.strategy import ops
    from gsplat.strategy.mcmc import MCMCStrategy
    return MCMCStrategy, ops


def scene(N, seed, alive_only=False):
    g = torch.Generator().manual_seed(seed)
    p = {
        "means": torch.randn(N, 3, generator=g),
        "scales": torch.rand(N, 3, generator=g) * 3.0 - 6.0,  # 0.0025 .. 0.05
        "quats": torch.randn(N, 4, generator=g),
        # logits across min_opacity = 0.005 (logit -5.29): ~13 % dead
        "opacities": (torch.rand(N, generator=g) * 4.0 - 1.0 if alive_only
                      else torch.randn(N, generator=g) * 3.0 - 2.0),
        "sh0": torch.randn(N, 1, 3, generator=g),
        "shN": torch.randn(N, 3, 3, generator=g) * 0.1,
    }
    return p, g


def run(name, N, seed, step, cap_max=1_000_000, lr=1.6e-4, alive_only=False):
    MCMCStrategy, ops = _import_reference()
    p, g = scene(N, seed, alive_only)
    params = {k: torch.nn.Parameter(v.clone()) for k, v in p.items()}
    opts = {k: torch.optim.Adam([{"params": params[k], "lr": 1e-3, "name": k}], eps=1e-15)
            for k in NAMES}
    for _ in range(2):  # populate the Adam moments
        for k in NAMES:
            params[k].grad = torch.randn(params[k].shape, generator=g) * 0.01
            opts[k].step()
            opts[k].zero_grad(set_to_none=True)
    before = {k: params[k].detach().clone() for k in NAMES}
    m0 = {k: opts[k].state[params[k]]["exp_avg"].clone() for k in NAMES}
    v0 = {k: opts[k].state[params[k]]["exp_avg_sq"].clone() for k in NAMES}

    draws, noise = [], []
    orig_sample, orig_randn_like = ops._multinomial_sample, torch.randn_like

    def rec_sample(weights, n, replacement=True):
        idx = orig_sample(weights, n, replacement)
        draws.append(idx.clone())
        return idx

    def rec_randn_like(t, *a, **kw):
        z = orig_randn_like(t, *a, **kw)
        noise.append(z.clone())
        return z

    strat = MCMCStrategy(cap_max=cap_max)
    state = strat.initialize_state()
    torch.manual_seed(2000 + seed)
    ops._multinomial_sample, torch.randn_like = rec_sample, rec_randn_like
    try:
        strat.step_post_backward(params, opts, state, step, info={}, lr=lr)
    finally:
        ops._multinomial_sample, torch.randn_like = orig_sample, orig_randn_like
    assert len(noise) == 1

    refine = step < strat.refine_stop_iter and step > strat.refine_start_iter \
        and step % strat.refine_every == 0
    n_dead = int((torch.sigmoid(before["opacities"]) <= strat.min_opacity).sum())
    reloc_idx = draws.pop(0) if refine and n_dead > 0 else torch.zeros(0, dtype=torch.int64)
    add_idx = draws.pop(0) if refine and draws else torch.zeros(0, dtype=torch.int64)
    assert not draws
    out = {"N": N, "step": step, "cap_max": cap_max, "lr": lr, "noise_lr": strat.noise_lr,
           "min_opacity": strat.min_opacity, "refine": int(refine), "n_dead": n_dead,
           "reloc_idx": reloc_idx.numpy(), "add_idx": add_idx.numpy(), "z": noise[0].numpy()}
    for k in NAMES:
        out[f"in_{k}"] = before[k].numpy()
        out[f"in_m_{k}"] = m0[k].numpy()
        out[f"in_v_{k}"] = v0[k].numpy()
        out[f"out_{k}"] = params[k].detach().numpy()
        out[f"out_m_{k}"] = opts[k].state[params[k]]["exp_avg"].numpy()
        out[f"out_v_{k}"] = opts[k].state[params[k]]["exp_avg_sq"].numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(name, "N", N, "->", len(params["means"]), "dead", n_dead, "relocated",
          len(reloc_idx), "added", len(add_idx))


CASES = {
    "mcmc_refine": dict(N=1000, seed=0, step=600),            # relocate + 5 % added + noise
    "mcmc_cap": dict(N=800, seed=1, step=700, cap_max=820),   # the add capped at cap_max
    "mcmc_alive": dict(N=600, seed=2, step=800, alive_only=True),  # nothing dead to relocate
    "mcmc_noise": dict(N=600, seed=3, step=601, lr=3e-4),     # not a refine step: noise only
}

if __name__ == "__main__":
    for name in (sys.argv[1:] or list(CASES)):
        run(name, **CASES[name])
