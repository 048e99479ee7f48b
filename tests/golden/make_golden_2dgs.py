"""Generate 2DGS projection golden vectors from the REFERENCE torch implementation.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden_2dgs.py

`gsplat.cuda._torch_impl_2dgs._fully_fused_projection_2dgs`
(gsplat/cuda/_torch_impl_2dgs.py:9-88) -- the function the reference's own
test compares its CUDA projection against (tests/test_2dgs.py:47-122) -- is
imported from /root/reference (package root stubbed so gsplat/__init__.py's
optional extras are not executed) and run on the CPU.  Outputs are stored in
the CUDA layout (ray_transforms permuted as tests/test_2dgs.py:69-71 does);
gradients come from torch autograd with seeded random cotangents, as in
tests/test_2dgs.py:87-104.  Scales[:, 2] = 1 as in the reference test: the
torch implementation scales the normal by s_z, the CUDA kernel does not.

Only the produced arrays are committed (.npz next to this script).
"""

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_ref():
    pkg = types.ModuleType("gsplat")
    pkg.__path__ = [os.path.join(REF, "gsplat")]
    sys.modules["gsplat"] = pkg
    from gsplat.cuda._torch_impl_2dgs import _fully_fused_projection_2dgs
    return _fully_fused_projection_2dgs


def reference_test_scene():
    """tests/test_2dgs.py:13-44 (4 surfels, 640x480)."""
    xs = torch.linspace(-1, 1, 2)
    xys = torch.stack(torch.meshgrid(xs, xs, indexing="ij"), dim=-1).reshape(-1, 2)
    means = torch.cat([xys, torch.ones_like(xys[:, :1]) * 3], dim=-1)
    quats = torch.tensor([[1.0, 0.0, 0.0, 0]]).repeat(len(means), 1)
    scales = torch.ones_like(means)
    scales[..., :2] *= 0.1
    viewmats = torch.eye(4).reshape(1, 4, 4)
    W, H = 640, 480
    Ks = torch.tensor([[W, 0.0, W // 2], [0.0, W, H // 2], [0.0, 0.0, 1.0]]).reshape(1, 3, 3)
    return means, quats, scales, viewmats, Ks, W, H


def random_scene(seed, N=400, C=2, W=256, H=192):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * 0.8
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.12 + 0.01
    scales[:, 2] = 1.0
    vms = []
    for c in range(C):
        a = 0.15 * c
        R = torch.tensor([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]],
                         dtype=torch.float32)
        vm = torch.eye(4)
        vm[:3, :3] = R
        vm[:3, 3] = torch.tensor([0.1 * c, -0.05 * c, 0.2 * c])
        vms.append(vm)
    viewmats = torch.stack(vms)
    Ks = torch.tensor([[220.0, 0, W / 2], [0, 210.0, H / 2], [0, 0, 1]]).expand(C, 3, 3).clone()
    return means, quats, scales, viewmats, Ks, W, H


def make(name, scene, fn, seed, zero_means2d_grad=False):
    means, quats, scales, viewmats, Ks, W, H = scene
    ins = [t.clone().requires_grad_(True) for t in (means, quats, scales)]
    radii, means2d, depths, rt, normals = fn(ins[0], ins[1], ins[2], viewmats, Ks, W, H)
    rt = rt.permute((0, 1, 3, 2))
    g = torch.Generator().manual_seed(seed)
    r = radii.float()
    v_means2d = torch.randn(means2d.shape, generator=g) * r[..., None]
    if zero_means2d_grad:  # isolates the exact part of the CUDA VJP
        v_means2d = torch.zeros_like(v_means2d)
    v_depths = torch.randn(depths.shape, generator=g) * r
    v_rt = torch.randn(rt.shape, generator=g) * r[..., None, None]
    v_normals = torch.randn(normals.shape, generator=g) * r[..., None]
    v_means, v_quats, v_scales = torch.autograd.grad(
        (means2d * v_means2d).sum() + (depths * v_depths).sum() + (rt * v_rt).sum()
        + (normals * v_normals).sum(), ins)
    np.savez_compressed(
        os.path.join(OUT, name), means=means.numpy(), quats=quats.numpy(), scales=scales.numpy(),
        viewmats=viewmats.numpy(), Ks=Ks.numpy(), width=W, height=H,
        radii=radii.numpy(), means2d=means2d.detach().numpy(), depths=depths.detach().numpy(),
        ray_transforms=rt.detach().numpy(), normals=normals.detach().numpy(),
        v_means2d=v_means2d.numpy(), v_depths=v_depths.numpy(), v_ray_transforms=v_rt.numpy(),
        v_normals=v_normals.numpy(), v_means=v_means.numpy(), v_quats=v_quats.numpy(),
        v_scales=v_scales.numpy())
    print(name, "radii>0:", int((radii > 0).sum()), "of", radii.numel())


def main():
    fn = _import_ref()
    make("proj2dgs_testdata.npz", reference_test_scene(), fn, seed=42)
    make("proj2dgs_random.npz", random_scene(1), fn, seed=7)
    make("proj2dgs_random_nomeans2d.npz", random_scene(2), fn, seed=8, zero_means2d_grad=True)


if __name__ == "__main__":
    main()
