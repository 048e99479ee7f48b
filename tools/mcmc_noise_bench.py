"""Time MCMC's per-step position noise: the fused HIP launch
(gsplat_hip.mcmc.inject_noise, one kernel on torch's normal draw) against the
reference's formulation in torch ops (gsplat/strategy/ops.py:343-369 with
the covariance from this backend's quat_scale_to_covar_preci launch), at the
Gaussian counts of BASELINE configs[1] / [2].  HIP events on the current
stream; prints one JSON line per size.

    python tools/mcmc_noise_bench.py [--iters 50]
"""

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))


def torch_noise(p, z, scaler):
    from gsplat_hip import quat_scale_to_covar_preci
    o = torch.sigmoid(p["opacities"].flatten())
    cov, _ = quat_scale_to_covar_preci(p["quats"], torch.exp(p["scales"]), compute_covar=True,
                                       compute_preci=False, triu=False)
    f = 1 / (1 + torch.exp(-100 * ((1 - o) - 0.995)))
    p["means"].add_(torch.einsum("bij,bj->bi", cov, z * f.unsqueeze(-1) * scaler))


def timed(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from gsplat_hip import mcmc
    gen = torch.Generator(device="cuda").manual_seed(0)
    for N in (1_006_065, 5_477_465):
        p = {"means": torch.randn(N, 3, device="cuda"), "quats": torch.randn(N, 4, device="cuda"),
             "scales": torch.rand(N, 3, device="cuda") * 4 - 6,
             "opacities": torch.randn(N, device="cuda") * 3 - 3}
        z = torch.randn(N, 3, device="cuda")
        ms_kernel = timed(lambda: mcmc.inject_noise(p, 1e-3, z=z), args.iters)
        ms_step = timed(lambda: mcmc.inject_noise(p, 1e-3, generator=gen), args.iters)
        ms_torch = timed(lambda: torch_noise(p, torch.randn(N, 3, device="cuda", generator=gen),
                                             1e-3), args.iters)
        byts = 68 * N  # means r+w, quats, log-scales, logit, z
        print(json.dumps({"N": N, "kernel_ms": round(ms_kernel, 4),
                          "kernel_GBps": round(byts / ms_kernel / 1e6, 1),
                          "hbm_frac": round(byts / ms_kernel / 1e6 / 8000.0, 3),
                          "with_randn_ms": round(ms_step, 4),
                          "torch_formula_ms": round(ms_torch, 4)}), flush=True)


if __name__ == "__main__":
    main()
