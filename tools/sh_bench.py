"""Time the fused SH colour kernels alone (fwd / bwd) at N Gaussians with a
given visible fraction; prints us per call."""
import sys

import torch

sys.path.insert(0, "gsplat-triton_amd")
import gsplat_hip  # noqa: E402
from gsplat_hip._wrapper import _SHColors  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_006_065
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
means = torch.randn(N, 3, device=dev, generator=g).requires_grad_(True)
sh0 = torch.randn(N, 1, 3, device=dev, generator=g).requires_grad_(True)
shN = torch.randn(N, 15, 3, device=dev, generator=g).requires_grad_(True)
vm = torch.eye(4, device=dev)[None].clone()
vm[0, 2, 3] = 5.0


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000


for frac in (0.0, 0.29, 1.0):
    radii = (torch.rand(1, N, device=dev, generator=g) < frac).int() * 3
    col = _SHColors.apply(3, means, vm, sh0, shN, radii)
    v = torch.randn_like(col)
    tf = timeit(lambda: _SHColors.apply(3, means, vm, sh0, shN, radii))
    tb = timeit(lambda: torch.autograd.grad(col, [means, sh0, shN], v, retain_graph=True))
    print(f"visible {frac:4.2f}: fwd {tf:7.1f} us   fwd+bwd-call {tb:7.1f} us")
