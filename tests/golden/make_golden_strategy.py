"""Golden vectors for DefaultStrategy's refine step from the REFERENCE's own
torch code: `DefaultStrategy._grow_gs` / `_prune_gs`
(gsplat/strategy/default.py:264-340) over `duplicate` / `split` / `remove` /
`reset_opa` (gsplat/strategy/ops.py:86-243) with real `torch.optim.Adam`
optimizers, run on the CPU.  Run in the build container only:

    python tests/golden/make_golden_strategy.py

Harness-only shims (nothing under /root/reference is modified or copied):
the `gsplat` package root is a stub (its __init__ pulls in the CUDA
extension), with `quat_scale_to_covar_preci` and `gsplat.relocation` (used
only by MCMC's relocate) as placeholders; `gsplat.utils` and the strategy
modules are the reference's.  The split noise is drawn by the reference from
the global CPU generator; the script re-draws it from the same seed and stores
it (`z`) so the HIP path can be fed the identical numbers.  Only arrays are
committed.
"""

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
NAMES = ("means", "scales", "quats", "opacities", "sh0", "shN")


def _import_reference():
    pkg = types.ModuleType("gsplat")
    pkg.__path__ = [os.path.join(REF, "gsplat")]
    pkg.quat_scale_to_covar_preci = None  # MCMC only
    sys.modules["gsplat"] = pkg
    reloc = types.ModuleType("gsplat.relocation")
    reloc.compute_relocation = None  # MCMC only
    sys.modules["gsplat.relocation"] = reloc
    from gsplat.strategy.default import DefaultStrategy
    from gsplat.strategy.ops import reset_opa
    return DefaultStrategy, reset_opa


def scene(N, seed):
    g = torch.Generator().manual_seed(seed)
    p = {
        "means": torch.randn(N, 3, generator=g),
        # log-uniform scales over [1e-3, 0.3]: both sides of grow_scale3d
        # (0.01) and prune_scale3d (0.1)
        "scales": torch.rand(N, 3, generator=g) * 5.7 - 6.9,
        "quats": torch.randn(N, 4, generator=g),
        # logits spread over the prune threshold sigmoid^-1(0.005) ~ -5.3
        "opacities": torch.randn(N, generator=g) * 3.0 - 2.0,
        "sh0": torch.randn(N, 1, 3, generator=g),
        "shN": torch.randn(N, 3, 3, generator=g) * 0.1,  # degree 1 keeps the file small
    }
    # running statistics: about a third above grow_grad2d = 2e-4 on average
    count = torch.randint(0, 6, (N,), generator=g).float()
    grad2d = torch.rand(N, generator=g) * 6e-4 * count
    return p, grad2d, count, g


def run(name, N, seed, step, scene_scale=1.0, revised=False, reset=False, scale2d_stop=0):
    DefaultStrategy, reset_opa = _import_reference()
    p, grad2d, count, g = scene(N, seed)
    params = {k: torch.nn.Parameter(v.clone()) for k, v in p.items()}
    opts = {k: torch.optim.Adam([{"params": params[k], "lr": 1e-3, "name": k}], eps=1e-15)
            for k in NAMES}
    # populate the Adam moments with two steps of random gradients
    for _ in range(2):
        for k in NAMES:
            params[k].grad = torch.randn(params[k].shape, generator=g) * 0.01
            opts[k].step()
            opts[k].zero_grad(set_to_none=True)
    before = {k: params[k].detach().clone() for k in NAMES}
    m0 = {k: opts[k].state[params[k]]["exp_avg"].clone() for k in NAMES}
    v0 = {k: opts[k].state[params[k]]["exp_avg_sq"].clone() for k in NAMES}

    strat = DefaultStrategy(revised_opacity=revised, refine_scale2d_stop_iter=scale2d_stop)
    state = {"grad2d": grad2d.clone(), "count": count.clone(), "scene_scale": scene_scale}
    radii = None
    if scale2d_stop > 0:
        # state["radii"] (max screen radius / max(W, H)) straddling
        # grow_scale2d = 0.05 and prune_scale2d = 0.15
        radii = torch.rand(N, generator=g) ** 3 * 0.25
        state["radii"] = radii.clone()
    torch.manual_seed(1000 + seed)
    n_dupli, n_split = strat._grow_gs(params, opts, state, step)
    n_prune = strat._prune_gs(params, opts, state, step)
    if reset:
        reset_opa(params=params, optimizers=opts, state=state, value=strat.prune_opa * 2.0)
    torch.manual_seed(1000 + seed)
    z = torch.randn(2, n_split, 3)  # the draw split() made (ops.py:147-152)

    out = {"N": N, "step": step, "scene_scale": scene_scale, "revised": int(revised),
           "reset": int(reset), "grad2d": grad2d.numpy(), "count": count.numpy(),
           "n_dupli": n_dupli, "n_split": n_split, "n_prune": n_prune, "z": z.numpy(),
           "scale2d_stop": scale2d_stop}
    if radii is not None:
        out["radii2d"] = radii.numpy()
    for k in NAMES:
        out[f"in_{k}"] = before[k].numpy()
        out[f"in_m_{k}"] = m0[k].numpy()
        out[f"in_v_{k}"] = v0[k].numpy()
        out[f"out_{k}"] = params[k].detach().numpy()
        out[f"out_m_{k}"] = opts[k].state[params[k]]["exp_avg"].numpy()
        out[f"out_v_{k}"] = opts[k].state[params[k]]["exp_avg_sq"].numpy()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(name, "N", N, "->", len(params["means"]), "dup", n_dupli, "split", n_split,
          "prune", n_prune)


CASES = {
    "densify_early": dict(N=1200, seed=0, step=600),                  # no size pruning (< 3000)
    "densify_late": dict(N=1200, seed=1, step=3100, scene_scale=1.3),  # + prune_scale3d
    "densify_revised": dict(N=1000, seed=2, step=3100, revised=True),
    "densify_reset": dict(N=1000, seed=3, step=6000, reset=True),      # refine then opacity reset
    # screen-size split / prune (refine_scale2d_stop_iter > 0, default.py:283-284, 325-326)
    "densify_scale2d": dict(N=1200, seed=4, step=3100, scale2d_stop=4000),
}

if __name__ == "__main__":
    # python make_golden_strategy.py [case ...]  (default: all)
    for name in (sys.argv[1:] or list(CASES)):
        run(name, **CASES[name])
