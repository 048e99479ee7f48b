"""One 3DGS training step over the HIP hot path (the unit bench.py measures).

Mirrors the per-iteration work of examples/simple_trainer.py with its default
config (sh_degree 3, packed=False, classic rasterize mode, batch 1):
  render (simple_trainer.py:453-507, 603-615) -> loss 0.8*L1 + 0.2*(1-SSIM,
  "valid" padding) (:642-646) -> backward (:683) -> DefaultStrategy running
  statistics (gsplat/strategy/default.py:213-262) -> Adam on every parameter
  group with the trainer's learning rates and batch scaling (:235-277).

model="2dgs" runs examples/simple_trainer_2dgs.py's default step instead:
rasterization_2dgs(render_mode="RGB+D") (simple_trainer_2dgs.py:549-563), the
same loss on the RGB channels (:590-594; normal/distortion losses are off by
default, :149-160), and the strategy statistics from meta["gradient_2dgs"]
(key_for_gradient, :307-311).

Multi-GPU is per-camera data parallelism: every rank holds the same
Gaussians and renders its own camera; the Gaussian gradients are summed over
RCCL/xGMI by reduce-scatter, each rank runs Adam on its share of the rows,
and the updated rows are all-gathered (distributed.ShardedAdam; the plain
per-group all-reduce + full Adam is `sharded_optimizer=False`).
"""

import math
import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .losses import FusedAdam, l1_ssim_loss
from .rendering import rasterization, rasterization_2dgs
from .strategy import activate, update_state_

C0 = 0.28209479177387814


def rgb_to_sh(rgb):
    return (rgb - 0.5) / C0


def load_garden_scene(path: str, scene_grid: int = 3):
    """load_test_data(scene_grid) semantics (gsplat/_helper.py:9-55) on the
    cropped garden fixture: tile the [-2,2]^3 crop into a scene_grid^2 grid."""
    d = np.load(path)
    means = torch.from_numpy(d["means3d"]).float()
    colors = torch.from_numpy(d["colors"].astype(np.float32) / 255.0)
    edges = torch.tensor([4.0, 4.0, 4.0])
    r = scene_grid // 2
    gx, gy = torch.meshgrid(torch.arange(-r, r + 1), torch.arange(-r, r + 1), indexing="ij")
    grid = torch.stack([gx, gy, torch.zeros_like(gx)], -1).reshape(-1, 3).float()
    means = (means[None] + grid[:, None] * edges).reshape(-1, 3)
    colors = colors.repeat(scene_grid ** 2, 1)
    return (means, colors, torch.from_numpy(d["viewmats"]), torch.from_numpy(d["Ks"]),
            int(d["width"]), int(d["height"]))


def camera_pool(viewmats, Ks, src_w, src_h, width, height, n, seed=0):
    """`n` cameras: the scene's own cameras first, then small jitters of them;
    intrinsics rescaled to width x height as profiling/main.py:85-87."""
    g = torch.Generator().manual_seed(seed)
    K = Ks.clone()
    K[:, 0, :] *= width / src_w
    K[:, 1, :] *= height / src_h
    vms, ks = [], []
    for i in range(n):
        v = viewmats[i % len(viewmats)].clone()
        if i >= len(viewmats):
            v[:3, 3] += torch.randn(3, generator=g) * 0.05
        vms.append(v)
        ks.append(K[i % len(K)])
    return torch.stack(vms), torch.stack(ks)


def _gauss_window(size=11, sigma=1.5, device="cpu"):
    x = torch.arange(size, dtype=torch.float32, device=device) - size // 2
    w = torch.exp(-(x ** 2) / (2 * sigma ** 2))
    return w / w.sum()


def ssim(img1, img2, window=None):
    """Mean SSIM with an 11x11 Gaussian window (sigma 1.5), "valid" padding --
    the quantity fused_ssim(..., padding="valid") returns. img: [B,C,H,W]."""
    Cc = img1.shape[1]
    w = _gauss_window(device=img1.device) if window is None else window
    wx = w.view(1, 1, 1, -1).repeat(Cc, 1, 1, 1)
    wy = w.view(1, 1, -1, 1).repeat(Cc, 1, 1, 1)

    def blur(x):
        return F.conv2d(F.conv2d(x, wx, groups=Cc), wy, groups=Cc)

    mu1, mu2 = blur(img1), blur(img2)
    s11 = blur(img1 * img1) - mu1 * mu1
    s22 = blur(img2 * img2) - mu2 * mu2
    s12 = blur(img1 * img2) - mu1 * mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1 * mu2 + C1) * (2 * s12 + C2)) / ((mu1 * mu1 + mu2 * mu2 + C1) * (s11 + s22 + C2))
    return m.mean()


class Trainer:
    """Holds the Gaussian parameters, Adam state and strategy statistics."""

    LRS = {"means": 1.6e-4, "scales": 5e-3, "quats": 1e-3, "opacities": 5e-2,
           "sh0": 2.5e-3, "shN": 2.5e-3 / 20}

    def __init__(self, points, rgbs, viewmats, Ks, width, height, sh_degree=3, device="cuda",
                 seed=42, world_size=1, rank=0, ssim_lambda=0.2, scene_scale=1.0,
                 fused=True, model="3dgs", sharded_optimizer=None):
        assert model in ("3dgs", "2dgs"), model
        self.model = model
        g = torch.Generator().manual_seed(seed)  # identical on every rank (replicas)
        N = points.shape[0]
        self.device = device
        self.width, self.height = width, height
        self.sh_degree = sh_degree
        self.ssim_lambda = ssim_lambda
        self.world_size, self.rank = world_size, rank
        # initial attributes as load_test_data(): scales U(0,0.02), unit quats,
        # opacities U(0,1); colours from the SfM points as SH DC terms.
        scales = torch.rand(N, 3, generator=g) * 0.02 + 1e-4
        quats = F.normalize(torch.randn(N, 4, generator=g), dim=-1)
        opac = torch.rand(N, generator=g).clamp(1e-3, 1 - 1e-3)
        K = (sh_degree + 1) ** 2
        sh = torch.zeros(N, K, 3)
        sh[:, 0, :] = rgb_to_sh(rgbs)
        sh[:, 1:, :] = torch.randn(N, K - 1, 3, generator=g) * 0.01
        self.params = {
            "means": points.clone(), "scales": torch.log(scales), "quats": quats,
            "opacities": torch.logit(opac), "sh0": sh[:, :1].contiguous(),
            "shN": sh[:, 1:].contiguous(),
        }
        self.params = {k: torch.nn.Parameter(v.to(device)) for k, v in self.params.items()}
        BS = world_size  # batch 1 per rank (simple_trainer.py:261-277)
        groups = [{"params": [p], "lr": self.LRS[k] * (scene_scale if k == "means" else 1.0)
                   * math.sqrt(BS), "name": k} for k, p in self.params.items()]
        kw = dict(eps=1e-15 / math.sqrt(BS), betas=(1 - BS * (1 - 0.9), 1 - BS * (1 - 0.999)))
        self.fused = fused
        # N > 1: gradients reduce-scattered, Adam on this rank's rows, rows
        # all-gathered (distributed.ShardedAdam) instead of all-reduce + full Adam
        # (None: when world_size > 1; True also at world_size 1, for tests)
        if sharded_optimizer is None:
            sharded_optimizer = world_size > 1
        self.sharded = fused and sharded_optimizer
        if self.sharded:
            from .distributed import ShardedAdam
            self.opt = ShardedAdam([g["params"][0] for g in groups], [g["lr"] for g in groups],
                                   **kw)
        elif fused:  # HIP loss + one-launch Adam (csrc/ssim.hip, csrc/adam.hip)
            self.opt = FusedAdam([g["params"][0] for g in groups], [g["lr"] for g in groups], **kw)
        else:  # torch reference path (conv SSIM, torch.optim.Adam)
            self.opt = torch.optim.Adam(groups, foreach=True, **kw)
        self.viewmats = viewmats.to(device)
        self.Ks = Ks.to(device)
        gt = torch.Generator().manual_seed(1234)
        self.targets = torch.rand(len(viewmats), height, width, 3, generator=gt).to(device)
        self.grad2d = torch.zeros(N, device=device)
        self.count = torch.zeros(N, device=device)
        self.window = _gauss_window(device=device)
        self.last_meta = None

    def camera_index(self, it: int) -> int:
        return (it * self.world_size + self.rank) % len(self.viewmats)

    def render(self, ci: int):
        p = self.params
        hook = None
        if self.sharded:
            # the previous step's all-gathers: geometry before the projection,
            # the SH rows only before the colours (evaluated after isect)
            names = list(self.params)
            self.opt.wait([names.index(k) for k in ("means", "scales", "quats", "opacities")])
            sh_idx = [names.index(k) for k in ("sh0", "shN")]
            hook = lambda: self.opt.wait(sh_idx)  # noqa: E731
        if self.fused:  # one HIP launch each way for both activations
            scales, opac = activate(p["scales"], p["opacities"])
        else:
            scales, opac = torch.exp(p["scales"]), torch.sigmoid(p["opacities"])
        if self.model == "2dgs":
            if hook is not None:
                hook()
            rc, ra, _, _, _, _, meta = rasterization_2dgs(
                p["means"], p["quats"], scales, opac, (p["sh0"], p["shN"]),
                self.viewmats[ci:ci + 1], self.Ks[ci:ci + 1], self.width, self.height,
                sh_degree=self.sh_degree, packed=False, near_plane=0.01, far_plane=1e10,
                render_mode="RGB+D")
            return rc[..., :3], ra, meta
        return rasterization(
            p["means"], p["quats"], scales, opac,
            (p["sh0"], p["shN"]) if self.fused else torch.cat([p["sh0"], p["shN"]], 1), self.viewmats[ci:ci + 1], self.Ks[ci:ci + 1],
            self.width, self.height, sh_degree=self.sh_degree, packed=False,
            near_plane=0.01, far_plane=1e10, radius_clip=0.0, rasterize_mode="classic",
            _colors_ready=hook)

    def step(self, it: int):
        ci = self.camera_index(it)
        colors, alphas, meta = self.render(ci)
        if self.model == "3dgs":
            meta["means2d"].retain_grad()  # DefaultStrategy.step_pre_backward
        gt = self.targets[ci:ci + 1]
        if self.fused:
            loss = l1_ssim_loss(colors, gt, self.ssim_lambda)
        else:
            l1 = F.l1_loss(colors, gt)
            ssim_loss = 1.0 - ssim(colors.permute(0, 3, 1, 2), gt.permute(0, 3, 1, 2),
                                   self.window)
            loss = l1 * (1.0 - self.ssim_lambda) + ssim_loss * self.ssim_lambda
        loss.backward()
        if self.world_size > 1 and not self.sharded:
            self.allreduce_grads()
        self.update_state(meta)
        if self.sharded:
            self.opt.step(defer_gather=True)
        else:
            self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        self.last_meta = meta
        return loss

    def allreduce_grads(self):
        """SUM the Gaussian gradients over ranks (RCCL over xGMI); issued
        largest-first so the long shN transfer starts earliest."""
        import torch.distributed as dist
        works = []
        for k in ("shN", "means", "quats", "scales", "sh0", "opacities"):
            gr = self.params[k].grad
            if gr is not None:
                works.append(dist.all_reduce(gr, op=dist.ReduceOp.SUM, async_op=True))
        for w in works:
            w.wait()

    @torch.no_grad()
    def update_state(self, meta):
        """DefaultStrategy._update_state for packed=False without the host
        sync of torch.where (default.py:213-262): same sums, masked."""
        g = meta["gradient_2dgs" if self.model == "2dgs" else "means2d"].grad
        if g is None:
            return
        if self.fused:
            update_state_(self.grad2d, self.count, g, meta["radii"], meta["width"],
                          meta["height"], meta["n_cameras"])
            return
        sx = meta["width"] / 2.0 * meta["n_cameras"]
        sy = meta["height"] / 2.0 * meta["n_cameras"]
        sel = meta["radii"] > 0  # [C, N]
        # elementwise hypot instead of a reduction over a size-2 dim
        nrm = torch.where(sel, torch.hypot(g[..., 0] * sx, g[..., 1] * sy), 0.0)
        if nrm.shape[0] == 1:
            self.grad2d.add_(nrm[0])
            self.count.add_(sel[0])
        else:
            self.grad2d.add_(nrm.sum(0))
            self.count.add_(sel.sum(0))
        # state["radii"] is only tracked when refine_scale2d_stop_iter > 0
        # (default 0, default.py:90,255-262)
