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

With `strategy=DefaultStrategyConfig()` the step also runs the reference's
DefaultStrategy schedule after the optimizer step (simple_trainer.py:808-826
-> gsplat/strategy/default.py:164-211): refine (grow + prune, one HIP
compaction of every parameter and both Adam moments, gsplat_hip.densify)
every `refine_every` steps in (refine_start_iter, refine_stop_iter), opacity
reset every `reset_every` steps.  `sh_degree_interval` enables the SH degree
schedule (simple_trainer.py:600), `max_steps` the means ExponentialLR
(:523-528), `init="sfm"` the SfM initialisation with knn scales, uniform
quaternions and init_opacity (:212-233).

With `strategy=MCMCStrategyConfig()` (gsplat_hip.mcmc) it runs MCMCStrategy
instead (simple_trainer.py:821-829 -> gsplat/strategy/mcmc.py:103-187): no
statistics; after the optimizer step, on refine steps the dead Gaussians are
relocated and 5 % are sampled in (up to cap_max), and every step the
positions get covariance-shaped noise (one fused HIP launch, its normal
draw made in the kernel from the trainer's key and the step) scaled by the
means learning rate of the next step.  With graph=True the steps between
refines are replays with the noise inside; the refines run eagerly.

Multi-GPU, two schemes, one process per GPU, every rank rendering its own
camera each step:
* `gaussian_shard=True` (the reference's multi-GPU training,
  simple_trainer.py:227-229,501 with gsplat/rendering.py:298-494): rank r
  holds the Gaussians [r::world] with their own Adam state and strategy
  statistics; the render is rasterization(distributed=True) -- the local
  Gaussians projected into every rank's camera, the projected pairs
  exchanged peer to peer over RCCL/xGMI, each rank rasterizing its camera
  with all Gaussians -- and the backward exchanges their gradients back, so
  each Gaussian's owner receives its gradient summed over all cameras.  No
  gradient all-reduce: per step a rank moves its shard's projected pairs
  (44 B each way per (Gaussian, camera)), not the whole scene's gradients.
  Densification runs per rank on its own shard, as the reference does.
* replicated (`sharded_optimizer`): every rank holds all Gaussians; the
  gradients are summed over RCCL/xGMI by reduce-scatter, each rank runs Adam
  on its share of the rows, and the updated rows are all-gathered
  (distributed.ShardedAdam; the plain per-group all-reduce + full Adam is
  `sharded_optimizer=False`).  Before a refine the densification statistics
  are summed over the ranks and the split noise comes from a generator seeded
  identically on every rank, so the replicas stay identical.
"""

import dataclasses
import math
import os
from typing import Dict, Optional, Union

import numpy as np
import torch
import torch.nn.functional as F

from . import densify
from .densify import DefaultStrategyConfig
from . import mcmc as _mcmc
from .mcmc import MCMCStrategyConfig
from .losses import FusedAdam, l1_ssim_loss, ssim_and_l1
from . import _wrapper
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


def knn_log_scales(points: torch.Tensor, init_scale: float = 1.0) -> torch.Tensor:
    """log of the RMS distance to the 3 nearest neighbours, repeated over the
    3 axes (simple_trainer.py:221-224 with examples/utils.py:141-151 knn):
    the SfM initialisation's scales.  One-off host work (a k-d tree)."""
    from scipy.spatial import cKDTree
    pts = points.detach().cpu().double().numpy()
    d, _ = cKDTree(pts).query(pts, k=4, workers=-1)
    dist2_avg = torch.from_numpy((d[:, 1:] ** 2).mean(-1)).float()
    return torch.log(torch.sqrt(dist2_avg) * init_scale).unsqueeze(-1).repeat(1, 3)


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


def _mean(x: torch.Tensor) -> torch.Tensor:
    """x.mean() as reductions that each give one output per workgroup: rows
    of 1024, then the row sums (and the tail).  torch's one-output reduction
    of a large tensor splits it over workgroups with a zero-filled semaphore
    buffer -- a memset node, which a captured step must not hold
    (graph_step.check_kernel_nodes_only) -- e.g. the regularisers of
    simple_trainer's mcmc preset at a million Gaussians."""
    x = x.reshape(-1)
    n = x.numel()
    q = n // 1024
    if q == 0:
        return x.sum() / n
    s = x[:q * 1024].view(q, 1024).sum(1).sum()
    if n > q * 1024:
        s = s + x[q * 1024:].sum()
    return s / n


class Trainer:
    """Holds the Gaussian parameters, Adam state and strategy statistics."""

    LRS = {"means": 1.6e-4, "scales": 5e-3, "quats": 1e-3, "opacities": 5e-2,
           "sh0": 2.5e-3, "shN": 2.5e-3 / 20}

    def __init__(self, points, rgbs, viewmats, Ks, width, height, sh_degree=3, device="cuda",
                 seed=42, world_size=1, rank=0, ssim_lambda=0.2, scene_scale=1.0,
                 fused=True, model="3dgs", sharded_optimizer=None,
                 strategy: Optional[Union[DefaultStrategyConfig, MCMCStrategyConfig]] = None,
                 sh_degree_interval: Optional[int] = None, max_steps: Optional[int] = None,
                 init: str = "random", init_opacity: float = 0.1, init_scale: float = 1.0,
                 targets: Optional[torch.Tensor] = None, opacity_reg: float = 0.0,
                 scale_reg: float = 0.0, dp_emulate_world: Optional[int] = None,
                 graph: bool = False, isect_capacity: Optional[int] = None,
                 gaussian_shard: bool = False, visible_adam: bool = False,
                 packed: bool = False, sparse_grad: bool = False, antialiased: bool = False):
        assert model in ("3dgs", "2dgs"), model
        assert init in ("random", "sfm"), init
        self.model = model
        g = torch.Generator().manual_seed(seed)  # identical on every rank (replicas)
        N = points.shape[0]
        self.device = device
        self.width, self.height = width, height
        self.sh_degree = sh_degree
        self.ssim_lambda = ssim_lambda
        self.world_size, self.rank = world_size, rank
        self.scene_scale = scene_scale
        # the caller's config object is not modified (a private copy)
        self.strategy = None if strategy is None else dataclasses.replace(strategy)
        # MCMCStrategy (mcmc.py): relocation / sample-add refines and the
        # per-step position noise instead of DefaultStrategy's statistics
        self.mcmc = isinstance(self.strategy, MCMCStrategyConfig)
        if self.mcmc:
            self._binoms = None  # initialize_state's table, on the device at first use
        elif self.strategy is not None and model == "2dgs":
            self.strategy.key_for_gradient = "gradient_2dgs"  # simple_trainer_2dgs.py:307-311
        # simple_trainer.py:135-137, 671-681: |sigmoid(opacities)| / |exp(scales)|
        # mean terms on the raw parameters (0 = off, the default config)
        self.opacity_reg, self.scale_reg = float(opacity_reg), float(scale_reg)
        self.sh_degree_interval = sh_degree_interval
        self.max_steps = max_steps
        K = (sh_degree + 1) ** 2
        sh = torch.zeros(N, K, 3)
        sh[:, 0, :] = rgb_to_sh(rgbs)
        if init == "random":
            # load_test_data(): scales U(0,0.02), unit quats, opacities U(0,1);
            # colours from the SfM points as SH DC terms
            scales = torch.log(torch.rand(N, 3, generator=g) * 0.02 + 1e-4)
            quats = F.normalize(torch.randn(N, 4, generator=g), dim=-1)
            opac = torch.logit(torch.rand(N, generator=g).clamp(1e-3, 1 - 1e-3))
            sh[:, 1:, :] = torch.randn(N, K - 1, 3, generator=g) * 0.01
        else:  # simple_trainer.create_splats_with_optimizers, init_type="sfm"
            scales = knn_log_scales(points, init_scale)
            quats = torch.rand(N, 4, generator=g)
            opac = torch.logit(torch.full((N,), float(init_opacity)))
        self.params = {
            "means": points.clone(), "scales": scales, "quats": quats, "opacities": opac,
            "sh0": sh[:, :1].contiguous(), "shN": sh[:, 1:].contiguous(),
        }
        # Gaussian-sharded: this rank's Gaussians [rank::world] of the scene
        # initialised as a whole (simple_trainer.py:221-229: knn scales over
        # all points, then the slice), so the shards together are the
        # one-GPU scene exactly
        self.gshard = bool(gaussian_shard)
        if self.gshard:
            assert model == "3dgs", "gaussian_shard: the 3DGS trainer"
            self.params = {k: v[rank::world_size].contiguous() for k, v in self.params.items()}
            self._n_world = [len(range(r, N, world_size)) for r in range(world_size)]
            N = self.params["means"].shape[0]
        self.params = {k: torch.nn.Parameter(v.float().contiguous().to(device))
                       for k, v in self.params.items()}
        BS = world_size  # batch 1 per rank (simple_trainer.py:261-277)
        self.lrs = [self.LRS[k] * (scene_scale if k == "means" else 1.0) * math.sqrt(BS)
                    for k in self.params]
        self.adam_kw = dict(eps=1e-15 / math.sqrt(BS),
                            betas=(1 - BS * (1 - 0.9), 1 - BS * (1 - 0.999)))
        self.fused = fused
        # simple_trainer.py:263-266,782-797 (cfg.visible_adam): SelectiveAdam --
        # the reference's Adam kernel (no bias correction) on the rows of the
        # Gaussians some camera of the step sees, (radii > 0).any(0); one
        # launch per group (gsplat_hip_selective_adam), no update fused into
        # a backward, steps issued eagerly
        self.visible_adam = bool(visible_adam)
        # simple_trainer.py:123,501 (cfg.packed): the render's [nnz] pairs
        # instead of [C, N] (rasterization(packed=True)); the strategy
        # statistics by index_add over meta["gaussian_ids"] (default.py:240-243);
        # steps issued eagerly
        self.packed = bool(packed)
        assert not (self.packed and (model != "3dgs" or gaussian_shard)), \
            "packed: the one-camera-per-rank 3DGS trainer"
        # simple_trainer.py:125,263-264,767-780 (cfg.sparse_grad): the packed
        # projection's COO gradients (rasterization(sparse_grad=True)), every
        # other gradient made COO over gaussian_ids, torch.optim.SparseAdam
        self.sparse_grad = bool(sparse_grad)
        # simple_trainer.py:129,482 (cfg.antialiased): rasterize_mode
        # "antialiased", the opacities scaled by the projection's compensation
        self.rasterize_mode = "antialiased" if antialiased else "classic"
        if self.sparse_grad:
            assert self.packed, "sparse_grad: packed mode only (simple_trainer.py:769)"
            assert world_size == 1, "sparse_grad: one rank"
        if self.visible_adam or self.sparse_grad:
            assert not (self.visible_adam and self.sparse_grad), "visible_adam or sparse_grad"
            assert not gaussian_shard and not sharded_optimizer, \
                "visible_adam: one rank or replicated ranks with all-reduced gradients"
            sharded_optimizer = False
        # N > 1: gradients reduce-scattered, Adam on this rank's rows, rows
        # all-gathered (distributed.ShardedAdam) instead of all-reduce + full Adam
        # (None: when world_size > 1; True also at world_size 1, for tests)
        if sharded_optimizer is None:
            sharded_optimizer = world_size > 1 and not self.gshard
        assert not (self.gshard and sharded_optimizer), "gaussian_shard: a local optimizer"
        self.sharded = fused and sharded_optimizer
        # measurement only (bench.py --dp-emulate W): one rank shards its
        # optimizer rows as W ranks would (ShardedAdam emulate_world)
        self.dp_emulate_world = dp_emulate_world if self.sharded else None
        # one rank, fused path: the SH coefficients' Adam step runs inside the
        # SH-colour backward (gsplat_hip_sh_colors_bwd_adam), so their
        # gradients never go through HBM; GSPLAT_HIP_SH_ADAM_IN_BWD=0 turns it off
        # (Gaussian-sharded too: the SH backward sums its shard's gradient over
        # every rank's camera in the kernel before the update)
        self.sh_adam_in_bwd = (fused and not self.sharded and not self.visible_adam
                               and not self.sparse_grad
                               and (world_size == 1 or self.gshard)
                               and os.environ.get("GSPLAT_HIP_SH_ADAM_IN_BWD", "1") != "0")
        # the exp / sigmoid VJPs and the means-gradient sum formed inside the
        # geometry groups' Adam (gsplat_hip_adam_step_ex): at one rank, and
        # under the sharded optimizer on the reduced shard (ShardedAdam.step)
        self.geom_fuse = (fused and not self.visible_adam and not self.sparse_grad
                          and (world_size == 1 or self.sharded or self.gshard)
                          and os.environ.get("GSPLAT_HIP_GEOM_FUSE", "1") != "0")
        # one rank: the geometry groups' whole Adam step inside the
        # projection backward (gsplat_hip_projection_bwd_adam, 2DGS:
        # gsplat_hip_projection_2dgs_bwd_adam), so their gradients never go
        # through HBM; GSPLAT_HIP_GEOM_IN_PROJ=0 turns it off.  Not with the
        # regularisers (extra terms on the raw parameters)
        self.geom_in_proj = (self.geom_fuse and world_size == 1 and not self.gshard
                             and not self.sharded and model in ("3dgs", "2dgs")
                             and self.opacity_reg == 0.0 and self.scale_reg == 0.0
                             and os.environ.get("GSPLAT_HIP_GEOM_IN_PROJ", "1") != "0")
        # sharded optimizer: the SH group's collectives on a communicator of
        # their own (issued from a gradient hook during the backward), the
        # geometry's on the default group
        self._sh_pg = None
        if self.sharded:
            import torch.distributed as dist
            self._sh_pg = dist.new_group(list(range(dist.get_world_size())))
        self._sh_ready = 0
        self.opt = self._make_optimizer(list(self.params.values()))
        self._register_hooks()
        self.viewmats = viewmats.to(device)
        self.Ks = Ks.to(device)
        if targets is None:
            gt = torch.Generator().manual_seed(1234)
            targets = torch.rand(len(viewmats), height, width, 3, generator=gt)
        self.targets = targets.to(device)
        self.grad2d = torch.zeros(N, device=device)
        self.count = torch.zeros(N, device=device)
        # state["radii"] (default.py:235-262): the largest screen radius of each
        # Gaussian normalised by max(W, H), tracked only while it is used
        self.radii2d = (torch.zeros(N, device=device) if self.strategy is not None
                        and getattr(self.strategy, "refine_scale2d_stop_iter", 0) > 0 else None)
        # split noise: the same stream on every rank (replicas stay identical);
        # Gaussian-sharded: a stream per shard
        self.rng = torch.Generator(device=device).manual_seed(
            seed + (7919 * rank if self.gshard else 0))
        # MCMC position noise: drawn in the noise kernel from this key and the
        # step (mcmc.inject_noise), so a replayed or re-run step draws the same
        self._noise_seed = ((seed + (7919 * rank if self.gshard else 0) + 1)
                            * 0x9E3779B97F4A7C15) % (1 << 64)
        self.window = _gauss_window(device=device)
        self.last_meta = None
        self.refine_log = []  # (step, n_dupli, n_split, n_prune, N after)
        # graph=True: the step as HIP graph replays where the configuration
        # allows (graph_step.graphable: fused one-rank 3DGS; with a
        # DefaultStrategy schedule the refines run eagerly between replays);
        # isect_capacity: its isect arrays' initial size (default: 1.25 x the
        # first camera's count)
        self._graph = None
        self.graph_fallback = None  # why the captured step fell back to eager, if it did
        if graph:
            from .graph_step import GraphStep, graphable
            if graphable(self):
                self._graph = GraphStep(self, capacity=isect_capacity)

    # ------------------------------------------------------------ optimizer
    def _make_optimizer(self, params):
        if self.sharded:
            from .distributed import ShardedAdam
            # geometry first: the next projection waits for it; the SH rows
            # only before the next step's colours (after its isect)
            names = list(self.params)
            groups = [[names.index(k) for k in ("means", "scales", "quats", "opacities")],
                      [names.index(k) for k in ("sh0", "shN")]]
            return ShardedAdam(params, self.lrs, groups=groups,
                               group_pgs=[None, getattr(self, "_sh_pg", None)],
                               emulate_world=getattr(self, "dp_emulate_world", None),
                               **self.adam_kw)
        groups = [{"params": [p], "lr": lr, "name": k}
                  for (k, p), lr in zip(self.params.items(), self.lrs)]
        if getattr(self, "visible_adam", False):
            from ._wrapper_aux import SelectiveAdam
            return SelectiveAdam(groups, **self.adam_kw)
        if getattr(self, "sparse_grad", False):
            return torch.optim.SparseAdam(groups, **self.adam_kw)
        if self.fused:  # HIP loss + one-launch Adam (csrc/ssim.hip, csrc/adam.hip)
            return FusedAdam(params, self.lrs, **self.adam_kw)
        return torch.optim.Adam(groups, foreach=True, **self.adam_kw)

    def _register_hooks(self):
        """Sharded optimizer: reduce-scatter the SH group as soon as the
        SH-colour backward has produced both of its gradients (the rest of
        the backward -- projection, activations -- is still to run), from a
        post-accumulate hook on sh0 and shN."""
        if not self.sharded:
            return
        for k in ("sh0", "shN"):
            self.params[k].register_post_accumulate_grad_hook(self._sh_grad_ready)

    def _sh_grad_ready(self, param):
        self._sh_ready += 1
        if self._sh_ready == 2:
            self.opt.reduce_early(1)

    def _set_means_lr(self, lr):
        if isinstance(self.opt, torch.optim.Optimizer):
            self.opt.param_groups[0]["lr"] = lr
        else:
            self.opt.lrs[0] = lr

    def moments(self):
        """name -> [exp_avg, exp_avg_sq] as full tensors shaped like the
        parameter (gathered over the ranks for the sharded optimizer)."""
        names = list(self.params)
        if self.sharded:
            return {k: list(mv) for k, mv in zip(names, self.opt.full_state())}
        if isinstance(self.opt, FusedAdam):
            self.sync()
            return {k: [self.opt.exp_avg[i], self.opt.exp_avg_sq[i]]
                    for i, k in enumerate(names)}
        out = {}
        for k in names:
            st = self.opt.state.get(self.params[k], {})
            if "exp_avg" not in st:  # no step taken yet
                z = torch.zeros_like(self.params[k])
                st = {"exp_avg": z, "exp_avg_sq": z.clone()}
            out[k] = [st["exp_avg"], st["exp_avg_sq"]]
        return out

    def _load_moments(self, moments):
        params = list(self.params.values())
        names = list(self.params)
        if self.sharded:
            step = self.opt.step_count
            self.opt = self._make_optimizer(params)
            self.opt.load_full_state([moments[k] for k in names], step)
        elif isinstance(self.opt, FusedAdam):
            self.opt.params = params
            self.opt.exp_avg = [moments[k][0] for k in names]
            self.opt.exp_avg_sq = [moments[k][1] for k in names]
        else:
            old = self.opt
            step = next(iter(old.state.values()), {}).get("step")
            lrs = [g["lr"] for g in old.param_groups]
            self.opt = self._make_optimizer(params)
            for g, lr in zip(self.opt.param_groups, lrs):
                g["lr"] = lr
            if step is not None:
                for k, p in self.params.items():
                    self.opt.state[p] = {"step": step.clone() if torch.is_tensor(step) else step,
                                         "exp_avg": moments[k][0],
                                         "exp_avg_sq": moments[k][1]}

    def sync(self):
        """Order the current stream after any optimizer communication still in
        flight (the sharded optimizer's deferred all-gathers): call before
        reading the parameters outside the training step (checkpoint, eval)."""
        if getattr(self, "_graph", None) is not None:
            self._graph.sync()
            if self._graph.failed is not None:  # a recovery's re-capture failed
                self.graph_fallback = self._graph.failed
                self._graph = None
        if self.sharded:
            self.opt.wait()

    def release_graph(self):
        """Stop replaying: settle the captured step's replays, destroy its
        graph (before destroy_process_group, see GraphStep.release) and issue
        later steps eagerly."""
        if getattr(self, "_graph", None) is not None:
            self._graph.release()
            self._graph = None

    def synced_params(self):
        self.sync()
        return self.params

    # ---------------------------------------------------------------- step
    def camera_index(self, it: int) -> int:
        return (it * self.world_size + self.rank) % len(self.viewmats)

    def sh_degree_at(self, it: int) -> int:
        if self.sh_degree_interval is None:
            return self.sh_degree
        return min(it // self.sh_degree_interval, self.sh_degree)

    def world_cameras(self, ci: int, world_ci=None):
        """Gaussian-sharded: the (viewmats, Ks) of every rank's camera, rank
        order -- the training schedule's (rank r renders (it*world + r) % n)
        or an explicit list `world_ci`."""
        n = len(self.viewmats)
        if world_ci is None:
            world_ci = [(ci - self.rank + r) % n for r in range(self.world_size)]
        key = tuple(int(c) for c in world_ci)
        cache = self.__dict__.setdefault("_wcam_cache", {})
        if key not in cache:
            if len(cache) > 4 * n:
                cache.clear()
            idx = torch.tensor(key, device=self.viewmats.device)
            cache[key] = (self.viewmats.index_select(0, idx), self.Ks.index_select(0, idx))
        return cache[key]

    def render(self, ci: int, sh_degree: Optional[int] = None,
               fusion: Optional[_wrapper.StepFusion] = None, world_ci=None):
        """Render camera `ci`; `fusion` (a training step's StepFusion) goes to
        the nodes whose backward hands their gradients to the optimizer.
        Gaussian-sharded: a collective -- every rank renders its own camera
        with all ranks' Gaussians (`world_ci`: see world_cameras)."""
        p = self.params
        deg = self.sh_degree if sh_degree is None else sh_degree
        hook = None
        if self.sharded:
            # the previous step's all-gathers: geometry before the projection,
            # the SH rows only before the colours (evaluated after isect)
            names = list(self.params)
            self.opt.wait([names.index(k) for k in ("means", "scales", "quats", "opacities")])
            sh_idx = [names.index(k) for k in ("sh0", "shN")]
            hook = lambda: self.opt.wait(sh_idx)  # noqa: E731
        if self.fused and not getattr(self, "sparse_grad", False):
            # one HIP launch each way for both activations (sparse_grad: torch's,
            # whose backward takes the projection's COO gradients)
            scales, opac = activate(p["scales"], p["opacities"], fusion)
        else:
            scales, opac = torch.exp(p["scales"]), torch.sigmoid(p["opacities"])
        absgrad = getattr(self.strategy, "absgrad", False)
        if self.model == "2dgs":
            if hook is not None:
                hook()
            rc, ra, _, _, _, _, meta = rasterization_2dgs(
                p["means"], p["quats"], scales, opac, (p["sh0"], p["shN"]),
                self.viewmats[ci:ci + 1], self.Ks[ci:ci + 1], self.width, self.height,
                sh_degree=deg, packed=False, near_plane=0.01, far_plane=1e10,
                render_mode="RGB+D", absgrad=absgrad, _fusion=fusion, _colors_only=True)
            meta["_rgbd"] = rc  # the loss reads its colour channels in place
            return rc[..., :3], ra, meta
        dkw = {}
        if getattr(self, "gshard", False):
            dkw = dict(distributed=True, _world_cameras=self.world_cameras(ci, world_ci),
                       _world_counts=self._n_world)
        with _wrapper.fwd_split(getattr(self, "split_div", None),
                                getattr(self, "split_threshold", None)):
            return rasterization(
                p["means"], p["quats"], scales, opac,
                (p["sh0"], p["shN"]) if self.fused else torch.cat([p["sh0"], p["shN"]], 1),
                self.viewmats[ci:ci + 1], self.Ks[ci:ci + 1], self.width, self.height,
                sh_degree=deg, packed=getattr(self, "packed", False), near_plane=0.01,
                far_plane=1e10, radius_clip=0.0, rasterize_mode=self.rasterize_mode,
                absgrad=absgrad,
                sparse_grad=getattr(self, "sparse_grad", False), _colors_ready=hook,
                _fusion=fusion, **dkw)

    def _tune_split(self, it: int):
        """Once, before the first step (and so before a graph capture freezes
        the forward's variant):
        * the split-forward threshold's divisor from the scene's termination.
          Pixels that rarely stop early (n_eff / n_isects > 0.75, M3: 0.89)
          make the heaviest tiles the forward's tail: split more of them
          (divisor 1100); scenes that terminate early (M2: 0.56) keep 550,
          whose split-capable variant would only cost occupancy.
          One-GPU 3DGS on the HIP path; GSPLAT_HIP_FWD_SPLIT_DIV set by the
          user wins;
        * which forward variant every render of this trainer launches: the
          split-capable one with this first render's threshold fixed if the
          render has a tile above it, else the plain one.  Decided once, so
          eager and captured steps run the same kernel with the same
          threshold (a captured step's isect count is its capacity) (the library's default heuristic reads an
          earlier render's largest tile from host-mapped memory with no sync:
          eager renders would pick a variant by timing).
        Both are this trainer's: its renders (and its graph capture) set them
        around their launches and restore the previous values
        (_wrapper.fwd_split), nothing else in the process sees them.  Costs
        one eager render (no backward) before the first step; a
        Gaussian-sharded render is a collective, and every rank's first step
        runs it."""
        self._split_tuned = True
        if self.model != "3dgs" or not self.fused:
            return
        colors, _, meta = self.render(self.camera_index(it), self.sh_degree_at(it))
        self.term_ratio = _wrapper.forward_termination_ratio(colors, meta, self.width, self.height)
        if self.world_size == 1 and not os.environ.get("GSPLAT_HIP_FWD_SPLIT_DIV"):
            self.split_div = 1100 if self.term_ratio > 0.75 else 550
        n = int(meta["isect_counts"][0]) if "isect_counts" in meta else meta["flatten_ids"].numel()
        with _wrapper.fwd_split(getattr(self, "split_div", None)):
            thr = _wrapper.fwd_split_threshold(n)
        self.max_tile_first = _wrapper.max_tile_isects(meta)
        self.split_launch = 1 if 0 <= thr < self.max_tile_first else 0
        # > 0: the split-capable forward at this fixed threshold; 0: never
        self.split_threshold = max(int(thr), 1) if self.split_launch else 0
        del colors, meta

    def step(self, it: int):
        if not getattr(self, "_split_tuned", False):
            self._tune_split(it)
        if getattr(self, "_graph", None) is not None:
            from .graph_step import GraphCaptureError
            try:
                loss = self._graph.step(it)
            except GraphCaptureError as e:
                # the capture failed (on any rank of a sharded job): eager
                # steps from here on, in this process (no re-exec); steps a
                # failed recovery voided have been re-run eagerly already
                import warnings
                self.graph_fallback = str(e)
                warnings.warn(f"gsplat_hip: {e}; issuing the training steps eagerly")
                self._graph = None
            else:
                if self.strategy is not None:
                    # eager refine / reset: drains the replays first
                    self.post_step(it, replayed=True)
                if self._graph is not None and self._graph.failed is not None:
                    self.graph_fallback = self._graph.failed  # (failed in that drain)
                    self._graph = None
                return loss
        loss = self._eager_step(it)
        if self.strategy is not None:
            self.post_step(it)
        return loss

    def _eager_step(self, it: int):
        """Training step `it` issued from the host (no refine / reset: post_step)."""
        ci = self.camera_index(it)
        self._sh_ready = 0
        if self.max_steps:  # means ExponentialLR: this step's lr, before the
            # backward that may run the geometry update (geom_in_proj)
            self._set_means_lr(self.lrs[0] * (0.01 ** (1.0 / self.max_steps)) ** it)
        fusion = self._make_fusion()
        colors, alphas, meta = self.render(ci, self.sh_degree_at(it), fusion)
        if self.model == "3dgs":
            # DefaultStrategy.step_pre_backward: the means2d gradient is
            # captured by a hook (retain_grad would clone it into .grad)
            meta["means2d"].register_hook(lambda g: meta.__setitem__("means2d_grad", g))
        gt = self.targets[ci:ci + 1]
        if self.fused and "_rgbd" in meta:  # 2DGS: the RGB+D render in place
            loss = l1_ssim_loss(meta["_rgbd"], gt, self.ssim_lambda, _channels=3)
        elif self.fused:
            loss = l1_ssim_loss(colors, gt, self.ssim_lambda)
        else:
            l1 = F.l1_loss(colors, gt)
            ssim_loss = 1.0 - ssim(colors.permute(0, 3, 1, 2), gt.permute(0, 3, 1, 2),
                                   self.window)
            loss = l1 * (1.0 - self.ssim_lambda) + ssim_loss * self.ssim_lambda
        loss = self._regularise(loss)
        if self.fused and loss.dim() == 0:
            # a constant 1.0 seed (no fill launch; the fused loss's backward
            # recognises it and skips its scaling launch)
            from . import losses as _losses
            if _losses.ONE_GRAD is None or _losses.ONE_GRAD.device != loss.device:
                _losses.ONE_GRAD = torch.ones((), device=loss.device)
            torch.autograd.backward(loss, _losses.ONE_GRAD)
        else:
            loss.backward()
        if self.world_size > 1 and not self.sharded and not getattr(self, "gshard", False):
            self.allreduce_grads()
        if self.strategy is None or (not self.mcmc and it < self.strategy.refine_stop_iter):
            self.update_state(meta)
        # whether this step's geometry update ran inside the projection backward
        self.geom_applied = bool(fusion is not None and fusion.geom_adam is not None
                                 and fusion.geom_adam.applied)
        if self.sharded:
            self.opt.step(defer_gather=True, xform=self._geom_xform(fusion))
        elif self.visible_adam:  # simple_trainer.py:782-797
            if meta.get("gaussian_ids") is not None:  # packed: the Gaussians of the pairs
                vis = torch.zeros(self.params["opacities"].shape[0], dtype=torch.bool,
                                  device=self.params["opacities"].device)
                vis[meta["gaussian_ids"]] = True
            else:  # (radii > 0).any(0)
                vis = meta["radii"] > 0
                if vis.dim() > 2:  # per-axis radii [C, N, 2]
                    vis = vis.all(-1)
                vis = vis.any(0)
            self.opt.step(vis)
        elif self.sparse_grad:  # simple_trainer.py:767-780, then SparseAdam
            ids = meta["gaussian_ids"]
            for k, p in self.params.items():
                g = p.grad
                if g is None or g.is_sparse:
                    continue
                p.grad = torch.sparse_coo_tensor(indices=ids[None], values=g[ids], size=p.size(),
                                                 is_coalesced=meta["n_cameras"] == 1)
            self.opt.step()
        else:
            self.opt.step(skip=self._sh_skip(fusion), xform=self._geom_xform(fusion))
        self.opt.zero_grad(set_to_none=True)
        self.last_meta = meta
        return loss

    def _regularise(self, loss):
        """simple_trainer.py:671-681: the opacity / scale regularisers on the raw
        parameters (their gradients reach .grad of the raw tensors through
        torch autograd; the fused optimizer adds them as extra terms)."""
        p = self.params
        if self.opacity_reg > 0.0:
            loss = loss + self.opacity_reg * _mean(torch.abs(torch.sigmoid(p["opacities"])))
        if self.scale_reg > 0.0:
            loss = loss + self.scale_reg * _mean(torch.abs(torch.exp(p["scales"])))
        return loss

    def _make_fusion(self) -> Optional[_wrapper.StepFusion]:
        """This step's StepFusion (None when nothing is fused): the SH groups'
        Adam inside the SH backward (sh_adam_in_bwd) and the geometry groups'
        gradient transforms inside their Adam (geom_fuse)."""
        fa = None
        if getattr(self, "sh_adam_in_bwd", False) and isinstance(self.opt, FusedAdam):
            names = list(self.params)
            i0, i1 = names.index("sh0"), names.index("shN")
            o = self.opt
            fa = _wrapper.ShAdamInBackward(
                self.params["sh0"].data, self.params["shN"].data, o.exp_avg[i0],
                o.exp_avg_sq[i0], o.exp_avg[i1], o.exp_avg_sq[i1], o.lrs[i0], o.lrs[i1],
                o.betas, o.eps, o.step_count + 1)
        geom = getattr(self, "geom_fuse", False) and (isinstance(self.opt, FusedAdam) or
                                                      self.sharded)
        ga = None
        if getattr(self, "geom_in_proj", False) and isinstance(self.opt, FusedAdam):
            ga = self.geom_adam_in_backward(self.opt.step_count + 1)
        if fa is None and not geom:
            return None
        return _wrapper.StepFusion(sh_adam=fa, geom=geom, geom_adam=ga)

    GEOM = ("means", "scales", "quats", "opacities")

    def geom_adam_in_backward(self, step, hyper=None, skip=None):
        """The geometry groups' Adam step for the projection backward
        (_wrapper.GeomAdamInBackward), in the trainer's group order."""
        names = list(self.params)
        o = self.opt
        ix = [names.index(k) for k in self.GEOM]
        return _wrapper.GeomAdamInBackward(
            [self.params[k].data for k in self.GEOM], [o.exp_avg[i] for i in ix],
            [o.exp_avg_sq[i] for i in ix], [o.lrs[i] for i in ix], o.betas, o.eps, step,
            hyper=hyper, skip=skip)

    def _sh_skip(self, fusion):
        """Indices of the groups whose update a backward already applied: the
        SH groups (SH-colour backward) and the geometry groups (projection
        backward).  Their .grad must then be empty: a loss term reaching them
        by another path would have been left out of that update."""
        if fusion is None:
            return ()
        names = list(self.params)
        done = []
        if fusion.sh_adam is not None and fusion.sh_adam.applied:
            done += [("sh0", "shN"), "GSPLAT_HIP_SH_ADAM_IN_BWD=0", "SH-colour"]
        if fusion.geom_adam is not None and fusion.geom_adam.applied:
            done += [self.GEOM, "GSPLAT_HIP_GEOM_IN_PROJ=0", "projection"]
        out = []
        for j in range(0, len(done), 3):
            keys, env, who = done[j:j + 3]
            for k in keys:
                if self.params[k].grad is not None:
                    raise RuntimeError(
                        f"{k} received a gradient outside the {who} backward while its Adam "
                        f"step was fused into that backward; set {env} for losses with extra "
                        "terms on those parameters")
            out += [names.index(k) for k in keys]
        return tuple(sorted(out))

    def _geom_xform(self, fusion):
        """FusedAdam xform of the gradients the fusion took: means = its .grad +
        the SH backward's part (autograd's sum), log-scales / logits = the exp
        / sigmoid VJPs of the activation backward formed in-register.  A
        gradient that also reached .grad of the raw log-scales / logits (a
        regulariser, simple_trainer.py:671-681) is added as an extra term:
        the VJP is then formed in torch with activate_bwd's operation order
        and summed with it, which is autograd's accumulation exactly."""
        if fusion is None or not fusion.geom:
            return None
        if fusion.geom_adam is not None and fusion.geom_adam.applied:
            return None  # the projection backward ran the geometry update
        names = list(self.params)
        xf = {}
        if fusion.v_dirs is not None:
            gm = self.params["means"].grad
            xf[names.index("means")] = (fusion.v_dirs, None, 0) if gm is None else \
                (gm, fusion.v_dirs, 1)
        if fusion.act_taken:
            for key, v, act, mode in (("scales", fusion.v_scales, fusion.scales, 2),
                                      ("opacities", fusion.v_opac, fusion.opac, 3)):
                if v is None:
                    continue  # that activation did not reach the loss
                extra = self.params[key].grad
                if extra is None:
                    xf[names.index(key)] = (v, act, mode)
                else:
                    vjp = v * act if mode == 2 else v * (1.0 - act) * act
                    xf[names.index(key)] = ((vjp + extra).contiguous(), None, 0)
        return xf or None

    # ---------------------------------------------------------------- eval
    @torch.no_grad()
    def evaluate(self, cameras=None, viewmats=None, Ks=None, images=None):
        """simple_trainer.py:854-932's eval metrics: render each camera,
        clamp to [0, 1], PSNR (data range 1) and SSIM (11x11 Gaussian, the
        fused "valid" SSIM of the loss) against the target, averaged.  Either
        indices into the trainer's camera pool / targets, or explicit
        viewmats [M,4,4], Ks [M,3,3] and images [M,H,W,3].  LPIPS is not
        computed (its network weights are a download)."""
        self.sync()
        if viewmats is None:
            idx = list(range(len(self.viewmats))) if cameras is None else list(cameras)
            viewmats, Ks, images = self.viewmats[idx], self.Ks[idx], self.targets[idx]
        psnrs, ssims = [], []
        saved = self.viewmats, self.Ks
        try:
            self.viewmats, self.Ks = viewmats.to(self.device), Ks.to(self.device)
            self.__dict__.pop("_wcam_cache", None)
            for i in range(len(viewmats)):
                # Gaussian-sharded: every rank renders camera i (a collective)
                colors, _, _ = self.render(i, world_ci=[i] * self.world_size)
                colors = torch.clamp(colors, 0.0, 1.0)
                gt = images[i:i + 1].to(self.device)
                mse = torch.mean((colors - gt) ** 2)
                psnrs.append(float(-10.0 * torch.log10(mse)))
                ssims.append(float(ssim_and_l1(colors, gt)[0]))
        finally:
            self.viewmats, self.Ks = saved
            self.__dict__.pop("_wcam_cache", None)
        return {"psnr": sum(psnrs) / len(psnrs), "ssim": sum(ssims) / len(ssims),
                "num_images": len(psnrs)}

    # ------------------------------------------------------------ strategy
    def post_step(self, it: int, replayed: bool = False):
        """DefaultStrategy.step_post_backward after the statistics
        (default.py:175-211): refine, then the opacity reset.  MCMC: its
        step_post_backward (mcmc_step); `replayed`: step `it` ran as a graph
        replay, which applied the position noise itself unless `it` refines."""
        cfg = self.strategy
        if self.mcmc:
            self.mcmc_step(it, noise=not (replayed and not cfg.is_refine_step(it)))
            return
        if it >= cfg.refine_stop_iter:
            return
        if cfg.is_refine_step(it):
            self.refine(it)
        if cfg.is_reset_step(it):
            self.reset_opacity()

    @torch.no_grad()
    def refine(self, it: int):
        self.sync()
        self.last_meta = None  # its tensors are sized for the old Gaussians
        if self.world_size > 1 and not getattr(self, "gshard", False):
            # every rank accumulated its own cameras: the batch statistics are
            # the sums (the screen radii: their maximum)
            import torch.distributed as dist
            works = [dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
                     for t in (self.grad2d, self.count)]
            if self.radii2d is not None:
                works.append(dist.all_reduce(self.radii2d, op=dist.ReduceOp.MAX, async_op=True))
            for w in works:
                w.wait()
        params = {k: p.data for k, p in self.params.items()}
        radii2d = self.radii2d if it < self.strategy.refine_scale2d_stop_iter else None
        new_p, new_m, counts = densify.refine(params, self.moments(), self.grad2d, self.count,
                                              it, self.strategy, self.scene_scale,
                                              generator=self.rng, radii2d=radii2d)
        self.params = {k: torch.nn.Parameter(v) for k, v in new_p.items()}
        self._load_moments(new_m)
        self._register_hooks()
        n = self.params["means"].shape[0]
        self.grad2d = torch.zeros(n, device=self.device)
        self.count = torch.zeros(n, device=self.device)
        if self.radii2d is not None:
            self.radii2d = torch.zeros(n, device=self.device)
        self.refine_log.append((it,) + tuple(counts) + (n,))
        self._param_gen = getattr(self, "_param_gen", 0) + 1  # a captured step re-captures
        if getattr(self, "gshard", False) and self.world_size > 1:  # each shard refined alone
            from .distributed import all_gather_int32
            self._n_world = all_gather_int32(self.world_size, n, device=self.device)

    @torch.no_grad()
    def mcmc_step(self, it: int, noise: bool = True):
        """MCMCStrategy.step_post_backward (mcmc.py:103-145) after step `it`'s
        optimizer update: on its refine steps relocate the dead Gaussians and
        sample in new ones (mcmc_refine), then the position noise (unless a
        graph replay of the step applied it)."""
        if self.strategy.is_refine_step(it):
            self.mcmc_refine(it)
        if noise:
            self.mcmc_noise(it)

    def mcmc_scaler(self, it: int) -> float:
        """The noise scale of step `it`: the means learning rate the reference
        passes (its scheduler already stepped, simple_trainer.py:808-829)
        times noise_lr (mcmc.py:143-145)."""
        lr = self.lrs[0]
        if self.max_steps:
            lr = lr * (0.01 ** (1.0 / self.max_steps)) ** (it + 1)
        return lr * self.strategy.noise_lr

    @torch.no_grad()
    def mcmc_noise(self, it: int):
        """inject_noise_to_position for step `it`, drawn in the kernel from
        (trainer key, it): the draw a graph replay of the step makes."""
        self.sync()
        _mcmc.inject_noise({k: p.data for k, p in self.params.items()}, self.mcmc_scaler(it),
                           seed=self._noise_seed, step=it)

    @torch.no_grad()
    def mcmc_refine(self, it: int):
        """_relocate_gs + _add_new_gs (mcmc.py:147-187) over the parameters and
        the Adam moments.  Gaussian-sharded: each shard alone, cap_max split
        evenly over the ranks."""
        cfg = self.strategy
        self.sync()
        self.last_meta = None
        if self._binoms is None:
            self._binoms = _mcmc.binoms(self.device)
        params = {k: p.data for k, p in self.params.items()}
        moms = self.moments()
        dead = torch.sigmoid(params["opacities"].flatten()) <= cfg.min_opacity
        n_reloc = _mcmc.relocate(params, moms, dead, self._binoms, cfg.min_opacity,
                                 generator=self.rng)
        gshard = getattr(self, "gshard", False) and self.world_size > 1
        cap = -(-cfg.cap_max // self.world_size) if gshard else cfg.cap_max
        n_add = _mcmc.n_to_add(params["means"].shape[0], cap)
        if n_add > 0:
            params, moms = _mcmc.sample_add(params, moms, n_add, self._binoms, cfg.min_opacity,
                                            generator=self.rng)
        self.params = {k: torch.nn.Parameter(v) for k, v in params.items()}
        self._load_moments(moms)
        self._register_hooks()
        n = self.params["means"].shape[0]
        self.grad2d = torch.zeros(n, device=self.device)
        self.count = torch.zeros(n, device=self.device)
        self.refine_log.append((it, n_reloc, n_add, n))
        if cfg.verbose:
            print(f"Step {it}: Relocated {n_reloc} GSs. Added {n_add} GSs. Now having {n} GSs.")
        self._param_gen = getattr(self, "_param_gen", 0) + 1
        if gshard:
            from .distributed import all_gather_int32
            self._n_world = all_gather_int32(self.world_size, n, device=self.device)

    @torch.no_grad()
    def reset_opacity(self):
        self.sync()
        value = self.strategy.prune_opa * 2.0
        if self.sharded:
            lim = float(torch.logit(torch.tensor(value, dtype=torch.float32)))
            self.params["opacities"].data.clamp_(max=lim)
            self.opt.zero_moments(list(self.params).index("opacities"))
        else:
            moms = self.moments()
            densify.reset_opacity({"opacities": self.params["opacities"].data},
                                  {"opacities": moms["opacities"]}, value)

    def densify_desc(self):
        if self.strategy is None:
            return "off (DefaultStrategy statistics only; fixed Gaussian count)"
        c = self.strategy
        if self.mcmc:
            return (f"MCMCStrategy relocate + add every {c.refine_every} steps in "
                    f"({c.refine_start_iter}, {c.refine_stop_iter}), cap {c.cap_max}, position "
                    f"noise every step (noise_lr {c.noise_lr:g}); refines so far "
                    f"(step, relocated, added, N): {self.refine_log}")
        return (f"DefaultStrategy refine every {c.refine_every} steps in "
                f"({c.refine_start_iter}, {c.refine_stop_iter}), opacity reset every "
                f"{c.reset_every}; refines so far: {self.refine_log}")

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
        sync of torch.where (default.py:213-262): same sums, masked; the
        screen-radius maximum of state["radii"] while refine_scale2d_stop_iter
        > 0 (default.py:255-262)."""
        if self.strategy is not None:
            key = self.strategy.key_for_gradient
        else:
            key = "gradient_2dgs" if self.model == "2dgs" else "means2d"
        if self.radii2d is not None:
            # radii / max(W, H) in float32 (int tensor / python float); the
            # reference's "should be scatter max" over the visible pairs --
            # invisible entries have radius 0 and leave the maximum unchanged
            r = meta["radii"].float() / float(max(meta["width"], meta["height"]))
            self.radii2d = torch.maximum(self.radii2d, r.amax(0))
        absgrad = getattr(self.strategy, "absgrad", False)
        if absgrad:
            g = meta[key].absgrad
        else:
            g = meta.get("means2d_grad") if key == "means2d" else None
            g = meta[key].grad if g is None else g
        if g is None:
            return
        if meta.get("gaussian_ids") is not None:  # packed: [nnz] pairs (default.py:240-254)
            ids = meta["gaussian_ids"]
            g = g.clone()
            g[..., 0] *= meta["width"] / 2.0 * meta["n_cameras"]
            g[..., 1] *= meta["height"] / 2.0 * meta["n_cameras"]
            self.grad2d.index_add_(0, ids, g.norm(dim=-1))
            self.count.index_add_(0, ids, torch.ones_like(ids, dtype=torch.float32))
            if self.radii2d is not None:
                self.radii2d[ids] = torch.maximum(
                    self.radii2d[ids],
                    meta["radii"].float() / float(max(meta["width"], meta["height"])))
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
