"""Time the one-launch Adam on the M2 parameter groups (1,006,065 Gaussians,
SH degree 3); prints us per step and the effective HBM bandwidth."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gsplat-triton_amd"))
from gsplat_hip.losses import FusedAdam  # noqa: E402

N = 1_006_065
shapes = [(N, 3), (N, 3), (N, 4), (N,), (N, 1, 3), (N, 15, 3)]
ps = [torch.randn(s, device="cuda").requires_grad_(True) for s in shapes]
for p in ps:
    p.grad = torch.randn_like(p)
opt = FusedAdam(ps, [1e-3] * len(ps), eps=1e-15)
for _ in range(3):
    opt.step()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
it = 50
for _ in range(it):
    opt.step()
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / it * 1000
nel = sum(p.numel() for p in ps)
print(f"variant {os.environ.get('GSPLAT_HIP_ADAM', '0')}: {us:.1f} us  {28 * nel / us / 1e3:.0f} GB/s")
