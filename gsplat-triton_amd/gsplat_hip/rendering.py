"""`rasterization()` front-end over the HIP backend.

Mirrors `gsplat.rendering.rasterization` (gsplat/rendering.py:44-598) for
the backend-independent torch glue: SH view directions, opacity repeat,
anti-aliasing compensation, RGB/D/ED channel assembly, channel chunking and
the `meta` dict consumed by the densification strategies.  The upstream file
is not modified in a drop-in deployment (it only needs the extra
`GSPLAT_BACKEND == "hip"` import branch); this copy exists so
the hot path can be exercised end to end without the rest of gsplat.
"""

import math
from typing import Callable, Dict, Optional, Tuple

import torch
from torch import Tensor

from . import _lib, _wrapper

# the captured 2DGS training step's tile culling of large surfels (ABI 34,
# gsplat_hip_isect_write_sorted_capped_surfel); a module attribute for A/B
TILE_CULL = True
from ._wrapper import (
    _dev_check,
    _f32c,
    _ptr,
    _stream,
    fully_fused_projection,
    isect_offset_encode,
    isect_tiles_begin,
    _rasterize_to_pixels,
    pack_render_records,
    rasterize_to_pixels,
    sh_colors,
    spherical_harmonics,
)


def _reshape_view(C: int, world_view: Tensor, N_world: list) -> Tensor:
    """[sum_i C*N_i, ...] blocks by source rank -> [C, sum_i N_i, ...]
    (gsplat/rendering.py:260-267).  One camera per rank: the blocks already
    are the Gaussians in rank order, a view (no copy)."""
    if C == 1:
        return world_view.unsqueeze(0)
    view_list = [x.split(int(x.shape[0] / C), dim=0)
                 for x in world_view.split([C * N_i for N_i in N_world], dim=0)]
    return torch.stack([torch.cat(parts, dim=0) for parts in zip(*view_list)], dim=0)


def rasterization(
    means: Tensor,  # [N, 3]
    quats: Tensor,  # [N, 4]
    scales: Tensor,  # [N, 3]
    opacities: Tensor,  # [N]
    colors: Tensor,  # [(C,) N, D] or [(C,) N, K, 3]
    viewmats: Tensor,  # [C, 4, 4]
    Ks: Tensor,  # [C, 3, 3]
    width: int,
    height: int,
    near_plane: float = 0.01,
    far_plane: float = 1e10,
    radius_clip: float = 0.0,
    eps2d: float = 0.3,
    sh_degree: Optional[int] = None,
    packed: bool = True,
    tile_size: int = 16,
    backgrounds: Optional[Tensor] = None,
    render_mode: str = "RGB",
    sparse_grad: bool = False,
    absgrad: bool = False,
    rasterize_mode: str = "classic",
    channel_chunk: int = 32,
    distributed: bool = False,
    camera_model: str = "pinhole",
    covars: Optional[Tensor] = None,
    _colors_ready: Optional[Callable[[], None]] = None,
    _fusion=None,
    _isect_capacity: Optional[int] = None,
    _isect_status: Optional[Tensor] = None,
    _isect_report=None,
    _world_cameras=None,
    _world_counts=None,
    _isect_ids: bool = True,
) -> Tuple[Tensor, Tensor, Dict]:
    """Rasterize N 3D Gaussians to C images (gsplat/rendering.py:44-598).

    Private arguments of the training harness (train_step.Trainer):
    `_colors_ready` (see below) and `_fusion`, a _wrapper.StepFusion handed
    to the fused SH-colour node (optimizer work folded into its backward);
    `_isect_capacity`: the sync-free tile intersection (no host read of
    n_isects, so the render can be captured into a HIP graph) into arrays of
    that many slots -- meta["isect_ids"] / ["flatten_ids"] are then
    capacity-sized, meta["isect_counts"] (device i64[4]: written, visible,
    overflow, n_isects) says how many are valid; an overflow also sets
    `_isect_status[0]` (sticky).  `_isect_report` = (host-mapped i64[ring][4]
    device pointer, device i64 slot): the counts also go to that ring row.
    distributed=True: `_world_cameras` = (viewmats, Ks) of every rank's
    cameras in rank order and `_world_counts` = every rank's Gaussian count,
    when the caller knows them (a trainer's camera schedule and shard sizes):
    the all-gathers of gsplat/rendering.py:303-308 -- one of them a host
    read -- are then skipped.  `_isect_ids=False` (with `_isect_capacity`,
    the training step): the sorted isects are emitted as depth ranks only
    when the rasterizer walks ranks -- meta["isect_ids"] / ["flatten_ids"]
    are then None (12 of 16 bytes per isect not written)."""
    meta = {}
    N = means.shape[0]
    C = viewmats.shape[0]
    device = means.device
    assert means.shape == (N, 3), means.shape
    if covars is None:
        assert quats.shape == (N, 4), quats.shape
        assert scales.shape == (N, 3), scales.shape
    else:
        assert covars.shape == (N, 3, 3), covars.shape
        raise NotImplementedError("covars input is not supported by this backend "
                                  "(same as the Triton backend, _wrapper.py:517-523)")
    assert opacities.shape == (N,), opacities.shape
    assert viewmats.shape == (C, 4, 4), viewmats.shape
    assert Ks.shape == (C, 3, 3), Ks.shape
    assert render_mode in ["RGB", "D", "ED", "RGB+D", "RGB+ED"], render_mode
    sh_rest = None
    if isinstance(colors, (tuple, list)):
        # extension: SH coefficients as the trainer stores them, (sh0 [N,1,3],
        # shN [N,K-1,3]); read in place instead of torch.cat per step
        assert sh_degree is not None, "a (sh0, shN) pair needs sh_degree"
        colors, sh_rest = colors
        assert colors.shape == (N, 1, 3) and sh_rest.shape[0] == N and sh_rest.shape[2] == 3, \
            (colors.shape, sh_rest.shape)
        assert (sh_degree + 1) ** 2 <= 1 + sh_rest.shape[1], sh_rest.shape
    elif sh_degree is None:
        assert (colors.dim() == 2 and colors.shape[0] == N) or (
            colors.dim() == 3 and colors.shape[:2] == (C, N)), colors.shape
    else:
        assert (colors.dim() == 3 and colors.shape[0] == N and colors.shape[2] == 3) or (
            colors.dim() == 4 and colors.shape[:2] == (C, N) and colors.shape[3] == 3), colors.shape
        assert (sh_degree + 1) ** 2 <= colors.shape[-2], colors.shape
    if absgrad:
        assert not distributed, "AbsGrad is not supported in distributed mode."
    if distributed:
        # Gaussian-sharded rendering (gsplat/rendering.py:298-310): project the
        # local Gaussians into every rank's cameras, exchange the projected
        # pairs, rasterize the local cameras
        from . import distributed as gdist
        assert (sh_degree is None and colors.dim() == 2) or (
            sh_degree is not None and (sh_rest is not None or colors.dim() == 3)), \
            "Distributed mode only supports per-Gaussian colors."
        world_rank, world_size = gdist.rank_world()
        if _world_counts is not None:
            N_world = [int(n) for n in _world_counts]
            assert len(N_world) == world_size and N_world[world_rank] == N, (N_world, N)
        else:
            N_world = gdist.all_gather_int32(world_size, N, device=device)
        C_world = [C] * world_size
        if _world_cameras is not None:
            vm_all, K_all = _world_cameras
            assert vm_all.shape == (C * world_size, 4, 4) and K_all.shape == (C * world_size, 3, 3)
            assert not viewmats.requires_grad, "_world_cameras: cameras without gradients"
            viewmats, Ks = vm_all, K_all
        else:
            viewmats, Ks = gdist.all_gather_tensor_list(world_size, [viewmats, Ks])
        C = len(viewmats)

    # a training step's geometry Adam inside the projection backward
    # (StepFusion.geom_adam): one camera, dense, no pose gradient
    geom_adam = (_fusion is not None and _fusion.geom_adam is not None and not packed
                 and not distributed and C == 1 and rasterize_mode == "classic"
                 and not viewmats.requires_grad)
    if geom_adam:
        proj = _wrapper._FullyFusedProjection.apply(
            means, None, quats, scales, viewmats, Ks, width, height, eps2d, near_plane,
            far_plane, radius_clip, False, camera_model, 256, _fusion)
    else:
        proj = fully_fused_projection(
            means, None, quats, scales, viewmats, Ks, width, height, eps2d=eps2d, packed=packed,
            near_plane=near_plane, far_plane=far_plane, radius_clip=radius_clip,
            sparse_grad=sparse_grad, calc_compensations=(rasterize_mode == "antialiased"),
            camera_model=camera_model)
    if packed:  # [nnz] pairs, all valid (gsplat/rendering.py:332-343)
        camera_ids, gaussian_ids, radii, means2d, depths, conics, compensations = proj
        opacities = opacities[gaussian_ids]
    else:
        radii, means2d, depths, conics, compensations = proj
        # [C, N]; for C == 1 a view, so backward is not a (copying) reduction
        if geom_adam:  # the same view, its gradient also handed to the fusion
            opacities = _wrapper._OpacityTap.apply(opacities, _fusion)
        else:
            opacities = opacities[None] if C == 1 else opacities.repeat(C, 1)
        camera_ids, gaussian_ids = None, None
    if compensations is not None:
        opacities = opacities * compensations
    meta.update({"camera_ids": camera_ids, "gaussian_ids": gaussian_ids, "radii": radii,
                 "means2d": means2d, "depths": depths, "conics": conics, "opacities": opacities})

    # tile intersection first: its counts travel to the host (the one sync of
    # the render) while the GPU computes the colours below
    tile_width = math.ceil(width / float(tile_size))
    tile_height = math.ceil(height / float(tile_size))
    pending_isects = None
    capped = _isect_capacity is not None
    if capped:  # Gaussian-sharded too: the isect of the exchanged pairs
        assert tile_size == 16 and not packed, "the sync-free isect: 16x16, packed=False"
    if not distributed:
        pending_isects = isect_tiles_begin(means2d, radii, depths, tile_size, tile_width,
                                           tile_height, packed=packed, n_cameras=C,
                                           camera_ids=camera_ids, gaussian_ids=gaussian_ids,
                                           sync=not capped)

    def eval_colors(colors):
        if packed:  # colours of the nnz pairs (gsplat/rendering.py:368-408)
            if sh_degree is None:
                colors = colors[gaussian_ids] if colors.dim() == 2 else colors[camera_ids, gaussian_ids]
            else:
                camtoworlds = torch.inverse(viewmats)
                dirs = means[gaussian_ids, :] - camtoworlds[camera_ids, :3, 3]
                if sh_rest is not None:
                    shs = (colors[gaussian_ids], sh_rest[gaussian_ids])
                elif colors.dim() == 3:
                    shs = colors[gaussian_ids]
                else:
                    shs = colors[camera_ids, gaussian_ids]
                colors = spherical_harmonics(sh_degree, dirs, shs, masks=radii > 0)
                colors = torch.clamp_min(colors + 0.5, 0.0)
        elif sh_degree is None:
            if colors.dim() == 2:
                colors = colors[None] if C == 1 else colors.expand(C, -1, -1)
        elif not viewmats.requires_grad and (sh_rest is not None or colors.dim() == 3):
            # one kernel each way: dirs from the camera centres, radii masking,
            # clamp_min(sh + 0.5, 0) (same values as the branch below)
            colors = sh_colors(sh_degree, means, viewmats,
                               colors if sh_rest is None else (colors, sh_rest), radii,
                               fusion=_fusion)
        else:
            camtoworlds = torch.inverse(viewmats)  # [C, 4, 4]
            dirs = means[None, :, :] - camtoworlds[:, None, :3, 3]  # [C, N, 3]
            masks = radii > 0
            # broadcast over cameras without copies (read in place by the SH
            # kernel); C == 1 uses an unsqueeze view so backward needs no reduction
            def bcast(x):
                return x[None] if C == 1 else x.expand(C, -1, -1, -1)
            shs = bcast(colors) if colors.dim() == 3 else colors
            if sh_rest is not None:
                shs = (shs, bcast(sh_rest))
            colors = spherical_harmonics(sh_degree, dirs, shs, masks=masks)  # [C, N, 3]
            colors = torch.clamp_min(colors + 0.5, 0.0)
        return colors

    # _colors_ready (private, bench harness): a callable run right before the
    # colours are evaluated, which are then evaluated after the tile
    # intersection -- lets a sharded optimizer's all-gather of the SH
    # coefficients overlap projection and isect (train_step.Trainer)
    late = _colors_ready is not None and not packed and not distributed
    if not late:
        if _colors_ready is not None:  # packed / distributed: wait before, not after
            _colors_ready()
        colors = eval_colors(colors)

    if distributed:  # gsplat/rendering.py:413-494
        if packed:
            cnts = torch.bincount(camera_ids, minlength=C).split(C_world, dim=0)
            cnts = [c.sum() for c in cnts]
            got = gdist.all_to_all_int32(world_size, cnts, device=device)
            (radii,) = gdist.all_to_all_tensor_list(world_size, [radii], cnts, output_splits=got)
            means2d, depths, conics, opacities, colors = gdist.all_to_all_tensor_list(
                world_size, [means2d, depths, conics, opacities, colors], cnts, output_splits=got)
            # camera ids global -> local, Gaussian ids local -> global
            reps = torch.stack(cnts)
            off = torch.cumsum(torch.tensor([0] + C_world[:-1], device=device,
                                            dtype=camera_ids.dtype), 0).repeat_interleave(reps)
            camera_ids = camera_ids - off
            off = torch.cumsum(torch.tensor([0] + N_world[:-1], device=device,
                                            dtype=gaussian_ids.dtype), 0).repeat_interleave(reps)
            gaussian_ids = gaussian_ids + off
            camera_ids, gaussian_ids = gdist.all_to_all_tensor_list(
                world_size, [camera_ids, gaussian_ids], cnts, output_splits=got)
            C = C_world[world_rank]
        elif C_world[world_rank] == 1:  # one camera per rank: one field-major exchange
            C = 1
            radii, means2d, depths, conics, opacities, colors = gdist.exchange_pairs(
                N_world, radii, means2d, depths, conics, opacities, colors)
        else:
            C = C_world[world_rank]
            splits = [C_i * N for C_i in C_world]
            outs = [C * N_i for N_i in N_world]
            (radii,) = gdist.all_to_all_tensor_list(world_size, [radii.flatten(0, 1)], splits=splits,
                                                    output_splits=outs)
            radii = _reshape_view(C, radii, N_world)
            parts = gdist.all_to_all_tensor_list(
                world_size, [means2d.flatten(0, 1), depths.flatten(0, 1), conics.flatten(0, 1),
                             opacities.flatten(0, 1), colors.flatten(0, 1)],
                splits=splits, output_splits=outs)
            means2d, depths, conics, opacities, colors = (_reshape_view(C, t, N_world)
                                                          for t in parts)
        pending_isects = isect_tiles_begin(means2d, radii, depths, tile_size, tile_width,
                                           tile_height, packed=packed, n_cameras=C,
                                           camera_ids=camera_ids, gaussian_ids=gaussian_ids,
                                           sync=not capped)

    def add_depth(colors, backgrounds):
        if render_mode in ["RGB+D", "RGB+ED"]:
            colors = torch.cat((colors, depths[..., None]), dim=-1)
            if backgrounds is not None:
                backgrounds = torch.cat([backgrounds, torch.zeros(C, 1, device=backgrounds.device)],
                                        -1)
        elif render_mode in ["D", "ED"]:
            colors = depths[..., None]
            if backgrounds is not None:
                backgrounds = torch.zeros(C, 1, device=backgrounds.device)
        return colors, backgrounds

    records = None
    ranked = pending_isects.will_rank(capped)
    if not late:
        colors, backgrounds = add_depth(colors, backgrounds)
        if colors.shape[-1] <= channel_chunk and not ranked:
            # queued before the isect sync, so the GPU has it to run while the
            # host waits for n_isects (rank-indexed records wait for the ranks)
            records = pack_render_records(means2d, conics, colors, opacities, tile_size,
                                          None if packed else pending_isects.tpg)

    counts = None
    if capped:
        # rank ids only: the rasterizer walks ranks through the render records
        ids = (_isect_ids or late or not _wrapper.RECORDS
               or opacities.numel() * 64 >= 2 ** 31)
        tiles_per_gauss, isect_ids, flatten_ids, counts = pending_isects.finish_capped(
            _isect_capacity, _isect_status, _isect_report, ids=ids)
        meta["isect_counts"] = counts
    else:
        tiles_per_gauss, isect_ids, flatten_ids = pending_isects.finish(sort=True)
    isect_offsets = pending_isects.offsets  # written with the sorted isects
    if isect_offsets is None:
        isect_offsets = isect_offset_encode(isect_ids, C, tile_width, tile_height,
                                            _n_isects_device=counts)
    ranks = pending_isects.ranks
    # the rasterizer's isect array: the flatten ids, or the rank ids it walks
    raster_ids = flatten_ids if flatten_ids is not None else ranks[0]
    if late:
        _colors_ready()
        colors, backgrounds = add_depth(eval_colors(colors), backgrounds)
    if (late or ranks is not None) and colors.shape[-1] <= channel_chunk:
        records = pack_render_records(means2d, conics, colors, opacities, tile_size,
                                      tiles_per_gauss, ranks)
    meta.update({"tile_width": tile_width, "tile_height": tile_height,
                 "tiles_per_gauss": tiles_per_gauss, "isect_ids": isect_ids,
                 "flatten_ids": flatten_ids, "isect_offsets": isect_offsets, "width": width,
                 "height": height, "tile_size": tile_size, "n_cameras": C})

    # only Gaussians with a tile are gathered: pack just their render records
    visible = None if packed else tiles_per_gauss
    if colors.shape[-1] > channel_chunk:
        n_chunks = (colors.shape[-1] + channel_chunk - 1) // channel_chunk
        render_colors, render_alphas = [], []
        for i in range(n_chunks):
            sl = slice(i * channel_chunk, (i + 1) * channel_chunk)
            rc, ra = _rasterize_to_pixels(
                means2d, conics, colors[..., sl], opacities, width, height, tile_size,
                isect_offsets, raster_ids,
                backgrounds=None if backgrounds is None else backgrounds[..., sl],
                packed=packed, absgrad=absgrad, visible=visible, n_isects_device=counts,
                ranks=ranks)
            render_colors.append(rc)
            render_alphas.append(ra)
        render_colors = torch.cat(render_colors, dim=-1)
        render_alphas = render_alphas[0]
    else:
        render_colors, render_alphas = _rasterize_to_pixels(
            means2d, conics, colors, opacities, width, height, tile_size, isect_offsets,
            raster_ids, backgrounds=backgrounds, packed=packed, absgrad=absgrad, visible=visible,
            records=records, n_isects_device=counts, ranks=ranks)
    if render_mode in ["ED", "RGB+ED"]:
        render_colors = torch.cat(
            [render_colors[..., :-1],
             render_colors[..., -1:] / render_alphas.clamp(min=1e-10)], dim=-1)
    return render_colors, render_alphas, meta


class _Rotate3(torch.autograd.Function):
    """_rotate's output for R = camtoworlds[C, :3, :3] and v [C, H, W, 3] in
    one HIP launch (gsplat_hip_rotate3); backward: autograd of the torch
    formula (only under a loss on the rendered normals)."""

    @staticmethod
    def forward(ctx, c2w, v):
        C = c2w.shape[0]
        vc = _f32c(v)
        out = torch.empty_like(vc)
        _lib.call("gsplat_hip_rotate3", C, vc.numel() // (3 * C), _ptr(_f32c(c2w)), _ptr(vc),
                  _ptr(out), _stream())
        ctx.save_for_backward(c2w, v)
        return out

    @staticmethod
    def backward(ctx, g):
        c2w, v = ctx.saved_tensors
        with torch.enable_grad():
            ins = [t.detach().requires_grad_(t.requires_grad) for t in (c2w, v)]
            out = _rotate(ins[0][..., :3, :3], ins[1])
            want = [t for t in ins if t.requires_grad]
            grads = iter(torch.autograd.grad(out, want, g, allow_unused=True)) if want else iter(())
        return tuple(next(grads) if t.requires_grad else None for t in ins)


def _rotate(R: Tensor, v: Tensor) -> Tensor:
    """out[..., i] = sum_j R[..., i, j] v[..., h, w, j] for R [..., 3, 3] and
    v [..., H, W, 3] -- the einsum "...ij,...hwj->...hwi" of the reference as
    three fused multiply-adds (the einsum lowers to a K=3 GEMM)."""
    Rt = R.transpose(-1, -2)[..., None, None, :, :]  # [..., 1, 1, 3(j), 3(i)]
    out = v[..., 0:1] * Rt[..., 0, :]
    out = torch.addcmul(out, v[..., 1:2], Rt[..., 1, :])
    return torch.addcmul(out, v[..., 2:3], Rt[..., 2, :])


def _depth_to_points(depths: Tensor, camtoworlds: Tensor, Ks: Tensor, z_depth: bool = True) -> Tensor:
    """Back-projects depth maps [..., H, W, 1] to world points (gsplat/utils.py:137-198)."""
    height, width = depths.shape[-3:-1]
    device = depths.device
    x, y = torch.meshgrid(torch.arange(width, device=device), torch.arange(height, device=device),
                          indexing="xy")
    fx, fy = Ks[..., 0, 0], Ks[..., 1, 1]
    cx, cy = Ks[..., 0, 2], Ks[..., 1, 2]
    camera_dirs = torch.nn.functional.pad(torch.stack(
        [(x - cx[..., None, None] + 0.5) / fx[..., None, None],
         (y - cy[..., None, None] + 0.5) / fy[..., None, None]], dim=-1), (0, 1), value=1.0)
    directions = _rotate(camtoworlds[..., :3, :3], camera_dirs)
    origins = camtoworlds[..., :3, -1]
    if not z_depth:
        directions = torch.nn.functional.normalize(directions, dim=-1)
    return origins[..., None, None, :] + depths * directions


def _depth_to_normal_torch(depths: Tensor, camtoworlds: Tensor, Ks: Tensor,
                           z_depth: bool = True) -> Tensor:
    """The formula of gsplat/utils.py:201-224 in torch ops (differentiated by
    _DepthToNormal.backward)."""
    points = _depth_to_points(depths, camtoworlds, Ks, z_depth=z_depth)
    dx = points[..., 2:, 1:-1, :] - points[..., :-2, 1:-1, :]
    dy = points[..., 1:-1, 2:, :] - points[..., 1:-1, :-2, :]
    normals = torch.nn.functional.normalize(torch.cross(dx, dy, dim=-1), dim=-1)
    return torch.nn.functional.pad(normals, (0, 0, 1, 1, 1, 1), value=0.0)


class _DepthToNormal(torch.autograd.Function):
    """Forward: one HIP launch (csrc/aux_ops.hip depth_to_normal_kernel)
    instead of a dozen full-image torch passes; backward (only when a loss
    uses the normals, e.g. the 2DGS normal-consistency term): autograd of the
    same formula in torch."""

    @staticmethod
    def forward(ctx, depths, camtoworlds, Ks, z_depth):
        _dev_check(depths, camtoworlds, Ks)
        H, W = depths.shape[-3:-1]
        lead = depths.shape[:-3]
        # the last channel of an RGB+D render is read in place (pixel stride)
        ps = depths.stride(-2)
        strided = (depths.dtype == torch.float32 and depths.shape[-1] == 1 and ps >= 1
                   and all(depths.stride(i) == depths.shape[i + 1] * depths.stride(i + 1)
                           for i in range(depths.dim() - 3)) and depths.stride(-3) == W * ps)
        d = depths if strided else _f32c(depths).reshape(-1, H, W)
        if not strided:
            ps = 1
        C = math.prod(lead) if lead else 1
        c2w = _f32c(camtoworlds).reshape(-1, 4, 4)
        k = _f32c(Ks).reshape(-1, 3, 3)
        assert c2w.shape[0] == C and k.shape[0] == C, (depths.shape, camtoworlds.shape, Ks.shape)
        out = torch.empty((C, H, W, 3), device=depths.device)
        _lib.call("gsplat_hip_depth_to_normal", C, H, W, _ptr(d), int(ps), _ptr(c2w), _ptr(k),
                  int(bool(z_depth)), _ptr(out), _stream())
        ctx.save_for_backward(depths, camtoworlds, Ks)
        ctx.z_depth = z_depth
        return out.reshape(*lead, H, W, 3)

    @staticmethod
    def backward(ctx, g):
        depths, camtoworlds, Ks = ctx.saved_tensors
        with torch.enable_grad():
            ins = [t.detach().requires_grad_(t.requires_grad)
                   for t in (depths, camtoworlds, Ks)]
            out = _depth_to_normal_torch(*ins, z_depth=ctx.z_depth)
            want = [t for t in ins if t.requires_grad]
            grads = iter(torch.autograd.grad(out, want, g, allow_unused=True)) if want else iter(())
        return tuple(next(grads) if t.requires_grad else None for t in ins) + (None,)


def depth_to_normal(depths: Tensor, camtoworlds: Tensor, Ks: Tensor, z_depth: bool = True) -> Tensor:
    """Surface normals from depth maps by central differences
    (gsplat/utils.py:201-224): depths [..., H, W, 1], camtoworlds [..., 4, 4],
    Ks [..., 3, 3] -> [..., H, W, 3]."""
    return _DepthToNormal.apply(depths, camtoworlds, Ks, z_depth)


def rasterization_2dgs(
    means: Tensor,  # [N, 3]
    quats: Tensor,  # [N, 4]
    scales: Tensor,  # [N, 3]
    opacities: Tensor,  # [N]
    colors: Tensor,  # [(C,) N, D] or [N, K, 3]
    viewmats: Tensor,  # [C, 4, 4]
    Ks: Tensor,  # [C, 3, 3]
    width: int,
    height: int,
    near_plane: float = 0.01,
    far_plane: float = 1e10,
    radius_clip: float = 0.0,
    eps2d: float = 0.3,
    sh_degree: Optional[int] = None,
    packed: bool = False,
    tile_size: int = 16,
    backgrounds: Optional[Tensor] = None,
    render_mode: str = "RGB",
    sparse_grad: bool = False,
    absgrad: bool = False,
    distloss: bool = False,
    depth_mode: str = "expected",
    _fusion=None,
    _isect_capacity: Optional[int] = None,
    _isect_status: Optional[Tensor] = None,
    _isect_report=None,
    _camtoworlds: Optional[Tensor] = None,
    _colors_only: bool = False,
):
    """Rasterize N surfels (2DGS) to C images (gsplat/rendering.py:1018-1339).

    Returns (render_colors, render_alphas, render_normals,
    render_normals_from_depth, render_distort, render_median, meta), with
    meta["gradient_2dgs"] the densification input whose .grad the 2DGS
    strategy reads.  Private (the captured training step, graph_step): the
    sync-free isect as rasterization()'s `_isect_capacity` / `_isect_status`
    / `_isect_report` (meta["isect_counts"]); `_camtoworlds` [C,4,4] the
    inverse viewmats (torch.linalg.inv reads its error flag on the host);
    `_colors_only` (the training step, whose loss reads the colours alone):
    render_normals and render_normals_from_depth are not formed (None) --
    the world-space rotation and the depth-to-normal pass are skipped."""
    from ._wrapper_2dgs import _SUPPORTED_D as _SUPPORTED_D_2DGS
    from ._wrapper_2dgs import fully_fused_projection_2dgs, rasterize_to_pixels_2dgs

    N = means.shape[0]
    C = viewmats.shape[0]
    assert means.shape == (N, 3), means.shape
    assert quats.shape == (N, 4), quats.shape
    assert scales.shape == (N, 3), scales.shape
    assert opacities.shape == (N,), opacities.shape
    assert viewmats.shape == (C, 4, 4), viewmats.shape
    assert Ks.shape == (C, 3, 3), Ks.shape
    assert render_mode in ["RGB", "D", "ED", "RGB+D", "RGB+ED"], render_mode
    if distloss:
        assert render_mode in ["D", "ED", "RGB+D", "RGB+ED"], (
            "distloss requires depth rendering, render_mode should be D, ED, RGB+D, RGB+ED, "
            f"but got {render_mode}")
    sh_rest = None
    if isinstance(colors, (tuple, list)):
        # extension (as rasterization()): SH coefficients as the trainer holds
        # them, (sh0 [N,1,3], shN [N,K-1,3]), read in place
        assert sh_degree is not None, "a (sh0, shN) pair needs sh_degree"
        colors, sh_rest = colors
        assert colors.shape == (N, 1, 3) and sh_rest.shape[0] == N and sh_rest.shape[2] == 3
        assert (sh_degree + 1) ** 2 <= 1 + sh_rest.shape[1], sh_rest.shape
    elif sh_degree is None:
        assert (colors.dim() == 2 and colors.shape[0] == N) or (
            colors.dim() == 3 and colors.shape[:2] == (C, N)), colors.shape
    else:
        assert colors.dim() == 3 and colors.shape[0] == N and colors.shape[2] == 3, colors.shape
        assert (sh_degree + 1) ** 2 <= colors.shape[1], colors.shape
    # a training step's geometry Adam inside the projection backward
    # (StepFusion.geom_adam, ABI 33): one camera, dense, no pose gradient
    geom_adam = (_fusion is not None and _fusion.geom_adam is not None and not packed
                 and C == 1 and not viewmats.requires_grad)
    if geom_adam:
        from ._wrapper_2dgs import _FullyFusedProjection2DGS
        proj = _FullyFusedProjection2DGS.apply(means, quats, scales, viewmats, Ks, width, height,
                                               eps2d, near_plane, far_plane, radius_clip, _fusion)
    else:
        proj = fully_fused_projection_2dgs(
            means, quats, scales, viewmats, Ks, width, height, eps2d, near_plane, far_plane,
            radius_clip, packed, sparse_grad)
    if packed:  # gsplat/rendering.py:1188-1199
        camera_ids, gaussian_ids, radii, means2d, depths, ray_transforms, normals = proj
        opacities = opacities[gaussian_ids]
    else:
        radii, means2d, depths, ray_transforms, normals = proj
        if geom_adam:  # the same view, its gradient also handed to the fusion
            opacities = _wrapper._OpacityTap.apply(opacities, _fusion)
        else:
            opacities = opacities[None] if C == 1 else opacities.repeat(C, 1)
        camera_ids, gaussian_ids = None, None
    # the densification input only receives a gradient (its values are never
    # read): the training step's (_colors_only) skips the reference's zero fill
    densify = (torch.empty_like(means2d, dtype=means.dtype) if _colors_only else
               torch.zeros_like(means2d, dtype=means.dtype)).requires_grad_(True)

    tile_width = math.ceil(width / float(tile_size))
    tile_height = math.ceil(height / float(tile_size))
    capped = _isect_capacity is not None
    assert not (capped and packed), "the sync-free isect: packed=False"
    pending_isects = isect_tiles_begin(means2d, radii, depths, tile_size, tile_width, tile_height,
                                       packed=packed, n_cameras=C, camera_ids=camera_ids,
                                       gaussian_ids=gaussian_ids, sync=not capped)

    if packed:  # gsplat/rendering.py:1216-1236
        if sh_degree is None:
            colors = colors[gaussian_ids] if colors.dim() == 2 else colors[camera_ids, gaussian_ids]
        else:
            shs = colors[gaussian_ids] if sh_rest is None else \
                (colors[gaussian_ids], sh_rest[gaussian_ids])
            dirs = means[gaussian_ids, :] - torch.inverse(viewmats)[camera_ids, :3, 3]
            colors = spherical_harmonics(sh_degree, dirs, shs, masks=radii > 0)
            colors = torch.clamp_min(colors + 0.5, 0.0)
    elif sh_degree is not None and not viewmats.requires_grad:
        # one kernel: dirs from -R^T t, radii masking, clamp_min(sh + 0.5, 0)
        colors = sh_colors(sh_degree, means, viewmats,
                           colors if sh_rest is None else (colors, sh_rest), radii,
                           fusion=_fusion)
    else:
        if sh_rest is not None:
            colors = torch.cat([colors, sh_rest], 1)
        if not (colors.dim() == 3 and sh_degree is None):
            colors = colors[None] if C == 1 else colors.expand(C, *([-1] * colors.dim()))
        if sh_degree is not None:
            camtoworlds = torch.inverse(viewmats)
            dirs = means[None, :, :] - camtoworlds[:, None, :3, 3]
            colors = spherical_harmonics(sh_degree, dirs, colors, masks=radii > 0)
            colors = torch.clamp_min(colors + 0.5, 0.0)

    depth_channel = None  # the rasterizer reads the depth channel in place (ABI 33)
    if (render_mode in ["RGB+D", "RGB+ED"] and not packed and backgrounds is None
            and colors.dim() == 3 and colors.shape[:2] == depths.shape
            and colors.shape[-1] + 1 in _SUPPORTED_D_2DGS):
        depth_channel = depths
    elif render_mode in ["RGB+D", "RGB+ED"]:
        colors = torch.cat((colors, depths[..., None]), dim=-1)
        if backgrounds is not None:
            backgrounds = torch.cat((backgrounds, torch.zeros((C, 1), device=colors.device)), -1)
    elif render_mode in ["D", "ED"]:
        colors = depths[..., None]

    # (the 2DGS rasterizer gathers its own arrays: no rank ids)
    counts = None
    if capped:
        # the training step (_colors_only) reads the offsets and flatten ids
        # only: no 64-bit isect ids (8 of 12 bytes per isect not written)
        # ... and, in the colours-only training step, large surfels' isects
        # only in the tiles their image can reach (the rasterizer culls the
        # others on every strip: same render, shorter isect list; ABI 34)
        tiles_per_gauss, isect_ids, flatten_ids, counts = pending_isects.finish_capped(
            _isect_capacity, _isect_status, _isect_report, ids=not _colors_only, ranks=False,
            surfel_cull=(ray_transforms, opacities) if (_colors_only and TILE_CULL) else None)
    else:
        tiles_per_gauss, isect_ids, flatten_ids = pending_isects.finish(sort=True, ranks=False)
    isect_offsets = pending_isects.offsets  # written with the sorted isects
    if isect_offsets is None:
        isect_offsets = isect_offset_encode(isect_ids, C, tile_width, tile_height)

    render_colors, render_alphas, render_normals, render_distort, render_median = \
        rasterize_to_pixels_2dgs(means2d, ray_transforms, colors, opacities, normals, densify,
                                 width, height, tile_size, isect_offsets, flatten_ids,
                                 backgrounds=backgrounds, packed=packed, absgrad=absgrad,
                                 distloss=distloss, _n_isects_device=counts,
                                 _visible=tiles_per_gauss, _colors_only=_colors_only,
                                 _depths=depth_channel)
    if _colors_only:
        meta = {"camera_ids": camera_ids, "gaussian_ids": gaussian_ids, "radii": radii,
                "means2d": means2d, "depths": depths, "ray_transforms": ray_transforms,
                "opacities": opacities, "normals": normals, "tile_width": tile_width,
                "tile_height": tile_height, "tiles_per_gauss": tiles_per_gauss,
                "isect_ids": isect_ids, "flatten_ids": flatten_ids,
                "isect_offsets": isect_offsets, "width": width, "height": height,
                "tile_size": tile_size, "n_cameras": C, "render_distort": render_distort,
                "gradient_2dgs": densify}
        if counts is not None:
            meta["isect_counts"] = counts
        return render_colors, render_alphas, None, None, render_distort, render_median, meta
    camtoworlds = torch.linalg.inv(viewmats) if _camtoworlds is None else _camtoworlds
    render_normals_from_depth = None
    if render_mode in ["ED", "RGB+ED"]:
        render_colors = torch.cat(
            [render_colors[..., :-1],
             render_colors[..., -1:] / render_alphas.clamp(min=1e-10)], dim=-1)
    if render_mode in ["RGB+ED", "RGB+D"]:
        if depth_mode == "expected":
            depth_for_normal = render_colors[..., -1:]
        elif depth_mode == "median":
            depth_for_normal = render_median
        render_normals_from_depth = depth_to_normal(
            depth_for_normal, camtoworlds, Ks).squeeze(0)

    meta = {"camera_ids": camera_ids, "gaussian_ids": gaussian_ids, "radii": radii,
            "means2d": means2d, "depths": depths, "ray_transforms": ray_transforms,
            "opacities": opacities, "normals": normals, "tile_width": tile_width,
            "tile_height": tile_height, "tiles_per_gauss": tiles_per_gauss,
            "isect_ids": isect_ids, "flatten_ids": flatten_ids, "isect_offsets": isect_offsets,
            "width": width, "height": height, "tile_size": tile_size, "n_cameras": C,
            "render_distort": render_distort, "gradient_2dgs": densify}
    if counts is not None:
        meta["isect_counts"] = counts
    if camtoworlds.dim() == 3 and render_normals.dim() == 4 and render_normals.is_cuda \
            and camtoworlds.shape[0] == render_normals.shape[0]:
        render_normals = _Rotate3.apply(camtoworlds, render_normals)
    else:
        render_normals = _rotate(camtoworlds[..., :3, :3], render_normals)
    return (render_colors, render_alphas, render_normals, render_normals_from_depth,
            render_distort, render_median, meta)
