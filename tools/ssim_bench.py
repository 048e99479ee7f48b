"""Time the training loss (l1_ssim_loss forward + backward) at 1080p RGB:
fused one-pass kernel vs the two-pass pair."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
from gsplat_hip.losses import l1_ssim_loss  # noqa: E402

fused = sys.argv[1] == "1"
g = torch.Generator(device="cuda").manual_seed(0)
base = torch.rand(1, 1080, 1922, 3, device="cuda", generator=g)
img = base[:, :, 2:].contiguous().requires_grad_(True)
gt = base[:, :, :-2].contiguous()


def run():
    loss = l1_ssim_loss(img, gt, 0.2, fused=fused)
    loss.backward()
    img.grad = None


for _ in range(10):
    run()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50):
    run()
b.record()
torch.cuda.synchronize()
loss = l1_ssim_loss(img, gt, 0.2, fused=fused)
loss.backward()
torch.cuda.synchronize()
# bit-level fingerprint: variants that only re-block the passes must agree
fp = (float(loss), float(img.grad.double().sum()), float(img.grad.abs().double().sum()))
print(f"fused={int(fused)}: "
      f"{a.elapsed_time(b) / 50 * 1e3:.1f} us per loss fwd+bwd; fingerprint {fp!r}")
