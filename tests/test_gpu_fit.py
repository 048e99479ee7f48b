"""Training sanity on the GPU: fitting a synthetic image with random
Gaussians (the reference's examples/image_fitting.py set-up: random means in
a box, a camera 8 units away, Adam on means/scales/quats/opacities/colours)
through the HIP path must converge, for 3DGS and 2DGS.  Quality evidence in
place of garden PSNR@7k (no dataset on the box)."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import gsplat_hip  # noqa: F401


def target(H, W):
    y, x = torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij")
    img = torch.stack([0.5 + 0.5 * torch.sin(6 * x), 0.5 + 0.5 * torch.cos(5 * y),
                       (x * y) ** 0.5], -1)
    img[: H // 2, : W // 2] = torch.tensor([1.0, 0.1, 0.1])
    return img.to(DEV)


def psnr(a, b):
    return float(-10 * torch.log10(((a - b) ** 2).mean()))


@pytest.mark.parametrize("model", ["3dgs", "2dgs"])
def test_image_fitting_converges(model):
    import gsplat_hip
    H = W = 96
    gt = target(H, W)
    g = torch.Generator(device=DEV).manual_seed(0)
    n = 4000
    means = (2 * (torch.rand(n, 3, device=DEV, generator=g) - 0.5)).requires_grad_(True)
    scales = (torch.rand(n, 3, device=DEV, generator=g) * -2 - 3).requires_grad_(True)
    quats = torch.randn(n, 4, device=DEV, generator=g).requires_grad_(True)
    opac = torch.zeros(n, device=DEV).requires_grad_(True)
    rgbs = torch.randn(n, 3, device=DEV, generator=g).requires_grad_(True)
    vm = torch.eye(4, device=DEV)
    vm[2, 3] = 8.0
    f = 0.5 * W / math.tan(0.25 * math.pi)
    K = torch.tensor([[f, 0, W / 2], [0, f, H / 2], [0, 0, 1]], device=DEV)
    opt = torch.optim.Adam([means, scales, quats, opac, rgbs], lr=0.01)
    fn = gsplat_hip.rasterization if model == "3dgs" else gsplat_hip.rasterization_2dgs
    first = None
    for it in range(300):
        out = fn(means, quats / quats.norm(dim=-1, keepdim=True), torch.exp(scales),
                 torch.sigmoid(opac), torch.sigmoid(rgbs), vm[None], K[None], W, H, packed=False)
        img = out[0][0]
        loss = ((img - gt) ** 2).mean()
        if first is None:
            first = psnr(img.detach(), gt)
        opt.zero_grad()
        loss.backward()
        opt.step()
    last = psnr(img.detach(), gt)
    print(f"{model}: PSNR {first:.2f} -> {last:.2f} dB after 300 steps")
    assert math.isfinite(last)
    assert last > first + 8.0 and last > 20.0, (model, first, last)
