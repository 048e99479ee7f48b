"""2DGS (surfel) ops backed by libgsplat_hip.so.

Drop-in for the 2DGS functions that `gsplat/rendering.py:31-34` imports from
`gsplat/cuda/_wrapper.py`:

    fully_fused_projection_2dgs  _wrapper.py:1229-1330 (autograd: _FullyFusedProjection2DGS :1333)
    rasterize_to_pixels_2dgs     _wrapper.py:1595-1726 (autograd: _RasterizeToPixels2DGS :1803)

Same signatures, defaults, assertions and autograd contract (argument order,
`None` gradients, `ctx.needs_input_grad[6]` gating of `v_backgrounds`,
`means2d.absgrad`, the `densify` input whose gradient is the densification
signal).  Every op runs through the HIP C ABI on torch's current stream; there
is no CPU fallback.
"""

import os
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._wrapper import _Timed, _aligned16, _dev_check, _f32c, _ptr, _stream


# ============================================================== projection ==
class _FullyFusedProjection2DGS(torch.autograd.Function):
    """Projects surfels to 2D (gsplat/cuda/_wrapper.py:1333-1437)."""

    @staticmethod
    def forward(ctx, means, quats, scales, viewmats, Ks, width, height, eps2d, near_plane,
                far_plane, radius_clip, fusion=None):
        # fusion: a training step's StepFusion whose geometry Adam this
        # backward runs (gsplat_hip_projection_2dgs_bwd_adam, one camera)
        ctx.fusion = fusion
        means, quats, scales, viewmats, Ks = (_f32c(x) for x in (means, quats, scales, viewmats, Ks))
        quats = _aligned16(quats)
        _dev_check(means, quats, scales, viewmats, Ks)
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device
        radii = torch.empty((C, N), dtype=torch.int32, device=dev)
        means2d = torch.empty((C, N, 2), dtype=torch.float32, device=dev)
        depths = torch.empty((C, N), dtype=torch.float32, device=dev)
        ray_transforms = torch.empty((C, N, 3, 3), dtype=torch.float32, device=dev)
        normals = torch.empty((C, N, 3), dtype=torch.float32, device=dev)
        _lib.call("gsplat_hip_projection_2dgs_fwd", C, N, _ptr(means), _ptr(quats), _ptr(scales),
                  _ptr(viewmats), _ptr(Ks), int(width), int(height), float(near_plane),
                  float(far_plane), float(radius_clip), _ptr(radii), _ptr(means2d),
                  _ptr(depths), _ptr(ray_transforms), _ptr(normals), _stream())
        ctx.save_for_backward(means, quats, scales, viewmats, Ks, radii, ray_transforms, normals)
        ctx.width, ctx.height, ctx.eps2d = int(width), int(height), eps2d
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # no zero-filled gradient of radii (or unused outputs)
        return radii, means2d, depths, ray_transforms, normals

    @staticmethod
    def backward(ctx, v_radii, v_means2d, v_depths, v_ray_transforms, v_normals):
        means, quats, scales, viewmats, Ks, radii, ray_transforms, normals = ctx.saved_tensors
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device

        def grad(t, shape):
            return torch.zeros(shape, device=dev) if t is None else _f32c(t)

        v_means2d = grad(v_means2d, (C, N, 2))
        v_ray_transforms = grad(v_ray_transforms, (C, N, 3, 3))
        # None (the rasterizer's normals had no gradient, ABI 33): null = zeros
        v_normals = None if v_normals is None else _f32c(v_normals)
        v_depths = None if v_depths is None else _f32c(v_depths)
        fusion = ctx.fusion
        if (fusion is not None and C == 1 and not ctx.needs_input_grad[3]
                and fusion.geom_adam_ready()):
            # the trainer's geometry Adam step in this backward: no gradients stored
            fusion.geom_adam.run_2dgs(means, quats, scales, viewmats, Ks, radii, ray_transforms,
                                      v_means2d, v_depths, v_normals, v_ray_transforms, fusion)
            return (None,) * 12
        v_means = torch.empty((N, 3), device=dev)
        v_quats = torch.empty((N, 4), device=dev)
        v_scales = torch.empty((N, 3), device=dev)
        v_viewmats = torch.empty((C, 4, 4), device=dev) if ctx.needs_input_grad[3] else None
        _lib.call("gsplat_hip_projection_2dgs_bwd", C, N, _ptr(means), _ptr(quats), _ptr(scales),
                  _ptr(viewmats), _ptr(Ks), ctx.width, ctx.height, _ptr(radii),
                  _ptr(ray_transforms), _ptr(v_means2d), _ptr(v_depths), _ptr(v_normals),
                  _ptr(v_ray_transforms), _ptr(v_means), _ptr(v_quats), _ptr(v_scales),
                  _ptr(v_viewmats), _stream())
        if not ctx.needs_input_grad[0]:
            v_means = None
        if not ctx.needs_input_grad[1]:
            v_quats = None
        if not ctx.needs_input_grad[2]:
            v_scales = None
        return (v_means, v_quats, v_scales, v_viewmats, None, None, None, None, None, None, None,
                None)


class _FullyFusedProjectionPacked2DGS(torch.autograd.Function):
    """Projects surfels to 2D, packed [nnz] outputs
    (gsplat/cuda/_wrapper.py:1440-1592).  One host read of nnz, as the
    reference's packed projection (its indptr / block_accum total)."""

    @staticmethod
    def forward(ctx, means, quats, scales, viewmats, Ks, width, height, near_plane, far_plane,
                radius_clip, sparse_grad):
        means, quats, scales, viewmats, Ks = (_f32c(x) for x in (means, quats, scales, viewmats, Ks))
        quats = _aligned16(quats)
        _dev_check(means, quats, scales, viewmats, Ks)
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device
        ws = torch.empty(max(int(_lib.query("gsplat_hip_projection_2dgs_packed_workspace_bytes",
                                            C, N)) // 8, 1), dtype=torch.int64, device=dev)
        nnz_dev = torch.empty(1, dtype=torch.int64, device=dev)
        args = (_ptr(means), _ptr(quats), _ptr(scales), _ptr(viewmats), _ptr(Ks), int(width),
                int(height), float(near_plane), float(far_plane), float(radius_clip))
        _lib.call("gsplat_hip_projection_2dgs_packed_count", C, N, *args, _ptr(ws),
                  _ptr(nnz_dev), _stream())
        nnz = int(nnz_dev.item())
        camera_ids = torch.empty(nnz, dtype=torch.int64, device=dev)
        gaussian_ids = torch.empty(nnz, dtype=torch.int64, device=dev)
        radii = torch.empty(nnz, dtype=torch.int32, device=dev)
        means2d = torch.empty((nnz, 2), device=dev)
        depths = torch.empty(nnz, device=dev)
        ray_transforms = torch.empty((nnz, 3, 3), device=dev)
        normals = torch.empty((nnz, 3), device=dev)
        _lib.call("gsplat_hip_projection_2dgs_packed_fwd", C, N, *args, _ptr(ws),
                  _ptr(camera_ids), _ptr(gaussian_ids), _ptr(radii), _ptr(means2d),
                  _ptr(depths), _ptr(ray_transforms), _ptr(normals), _stream())
        ctx.save_for_backward(camera_ids, gaussian_ids, means, quats, scales, viewmats, Ks,
                              ray_transforms)
        ctx.width, ctx.height, ctx.sparse_grad = int(width), int(height), sparse_grad
        ctx.mark_non_differentiable(camera_ids, gaussian_ids, radii)
        return camera_ids, gaussian_ids, radii, means2d, depths, ray_transforms, normals

    @staticmethod
    def backward(ctx, v_camera_ids, v_gaussian_ids, v_radii, v_means2d, v_depths,
                 v_ray_transforms, v_normals):
        camera_ids, gaussian_ids, means, quats, scales, viewmats, Ks, ray_transforms = \
            ctx.saved_tensors
        C, N, nnz = viewmats.shape[0], means.shape[0], camera_ids.numel()
        dev = means.device

        def g(t, shape):
            return torch.zeros(shape, device=dev) if t is None else _f32c(t)

        v_means2d = g(v_means2d, (nnz, 2))
        v_ray_transforms = g(v_ray_transforms, (nnz, 3, 3))
        v_normals = g(v_normals, (nnz, 3))
        v_depths = None if v_depths is None else _f32c(v_depths)
        rows = nnz if ctx.sparse_grad else N
        v_means = torch.empty((rows, 3), device=dev)
        v_quats = torch.empty((rows, 4), device=dev)
        v_scales = torch.empty((rows, 3), device=dev)
        v_viewmats = torch.empty((C, 4, 4), device=dev) if ctx.needs_input_grad[3] else None
        _lib.call("gsplat_hip_projection_2dgs_packed_bwd", C, N, nnz, _ptr(means), _ptr(quats),
                  _ptr(scales), _ptr(viewmats), _ptr(Ks), ctx.width, ctx.height,
                  _ptr(camera_ids), _ptr(gaussian_ids), _ptr(ray_transforms), _ptr(v_means2d),
                  _ptr(v_depths), _ptr(v_normals), _ptr(v_ray_transforms),
                  int(bool(ctx.sparse_grad)), _ptr(v_means), _ptr(v_quats), _ptr(v_scales),
                  _ptr(v_viewmats), _stream())
        if ctx.sparse_grad:  # COO gradients (_wrapper.py:1529-1570)
            def coo(v, like):
                return torch.sparse_coo_tensor(indices=gaussian_ids[None], values=v,
                                               size=like.size(), is_coalesced=C == 1)
            v_means, v_quats, v_scales = coo(v_means, means), coo(v_quats, quats), \
                coo(v_scales, scales)
        return (v_means if ctx.needs_input_grad[0] else None,
                v_quats if ctx.needs_input_grad[1] else None,
                v_scales if ctx.needs_input_grad[2] else None,
                v_viewmats, None, None, None, None, None, None, None)


def fully_fused_projection_2dgs(
    means: Tensor,  # [N, 3]
    quats: Tensor,  # [N, 4]
    scales: Tensor,  # [N, 3]
    viewmats: Tensor,  # [C, 4, 4]
    Ks: Tensor,  # [C, 3, 3]
    width: int,
    height: int,
    eps2d: float = 0.3,
    near_plane: float = 0.01,
    far_plane: float = 1e10,
    radius_clip: float = 0.0,
    packed: bool = False,
    sparse_grad: bool = False,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Ray-splat transforms, 2D means, depths, radii and normals of surfels
    (gsplat/cuda/_wrapper.py:1229-1330).  Returns (radii i32[C,N],
    means2d[C,N,2], depths[C,N], ray_transforms[C,N,3,3], normals[C,N,3]), or
    with packed=True (camera_ids i64[nnz], gaussian_ids i64[nnz], radii
    i32[nnz], means2d[nnz,2], depths[nnz], ray_transforms[nnz,3,3],
    normals[nnz,3])."""
    C = viewmats.size(0)
    N = means.size(0)
    assert means.size() == (N, 3), means.size()
    assert viewmats.size() == (C, 4, 4), viewmats.size()
    assert Ks.size() == (C, 3, 3), Ks.size()
    means = means.contiguous()
    assert quats is not None, "quats is required"
    assert scales is not None, "scales is required"
    assert quats.size() == (N, 4), quats.size()
    assert scales.size() == (N, 3), scales.size()
    quats = quats.contiguous()
    scales = scales.contiguous()
    if sparse_grad:
        assert packed, "sparse_grad is only supported when packed is True"
    viewmats = viewmats.contiguous()
    Ks = Ks.contiguous()
    if packed:
        return _FullyFusedProjectionPacked2DGS.apply(means, quats, scales, viewmats, Ks, width,
                                                     height, near_plane, far_plane, radius_clip,
                                                     sparse_grad)
    return _FullyFusedProjection2DGS.apply(means, quats, scales, viewmats, Ks, width, height,
                                           eps2d, near_plane, far_plane, radius_clip)


# ============================================================ rasterization ==
_SUPPORTED_D = (1, 2, 3, 4, 5, 6, 7, 8, 9, 16, 17, 32, 33)
# the forward composites from scalar-operand records (csrc/surfel.hip
# fwd2s_kernel) where the configuration has them
# (GSPLAT_HIP_SURFEL_SREC=0: the LDS-queue forward, fwd2_kernel)
SREC = os.environ.get("GSPLAT_HIP_SURFEL_SREC", "1") != "0"
# heaviest-first dispatch order of the tiles, forward and backward
# (M5: 293 -> 309 images/s, backward 1.68 -> 1.48 ms; GSPLAT_HIP_SURFEL_ORDER=0 turns it off)
ORDER = os.environ.get("GSPLAT_HIP_SURFEL_ORDER", "1") != "0"


class _RasterizeToPixels2DGS(torch.autograd.Function):
    """Surfel rasterizer (gsplat/cuda/_wrapper.py:1803-1971)."""

    @staticmethod
    def forward(ctx, means2d, ray_transforms, colors, opacities, normals, densify, backgrounds,
                masks, width, height, tile_size, isect_offsets, flatten_ids, absgrad, distloss,
                n_dev=None, visible=None, colors_only=False, depths=None):
        # depths (ABI 33, [C, N] or [nnz], or None): the last colour channel,
        # read in place -- colors then holds the other D - 1
        means2d, ray_transforms, colors, opacities, normals, backgrounds, depths = (
            _f32c(x) for x in (means2d, ray_transforms, colors, opacities, normals, backgrounds,
                               depths))
        _dev_check(means2d, ray_transforms, colors, opacities, normals, isect_offsets, flatten_ids)
        C, th, tw = isect_offsets.shape
        D = colors.shape[-1] + (1 if depths is not None else 0)
        dev = means2d.device
        isect_offsets = isect_offsets.to(torch.int32).contiguous()
        flatten_ids = flatten_ids.to(torch.int32).contiguous()
        masks_u8 = None if masks is None else masks.to(torch.uint8).contiguous()
        records = None
        nf = int(_lib.query("gsplat_hip_rasterize_2dgs_record_floats", D, int(tile_size))) \
            if SREC else 0
        # colours-only (ABI 33, the record path): no normals / distortion /
        # median images (None) and no median ids
        lean = bool(colors_only) and nf > 0
        render_colors = torch.empty((C, height, width, D), device=dev)
        render_alphas = torch.empty((C, height, width, 1), device=dev)
        last_ids = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        render_normals = render_distort = render_median = median_ids = None
        if not lean:
            render_normals = torch.empty((C, height, width, 3), device=dev)
            render_distort = torch.empty((C, height, width, 1), device=dev)
            render_median = torch.empty((C, height, width, 1), device=dev)
            median_ids = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        if nf:  # scalar-operand records (GSPLAT_HIP_SURFEL_SREC=1)
            G = opacities.numel()
            records = torch.empty(max(G, 1) * nf, device=dev)
            _lib.call("gsplat_hip_rasterize_2dgs_pack_records", G, D, _ptr(means2d),
                      _ptr(ray_transforms), _ptr(opacities), _ptr(normals), _ptr(colors),
                      _ptr(depths), _ptr(visible), _ptr(records), _stream())
        order = torch.empty(C * th * tw, dtype=torch.int32, device=dev) \
            if ORDER and int(tile_size) == 16 else None
        with _Timed("rasterize_2dgs_fwd"):
            _lib.call("gsplat_hip_rasterize_2dgs_fwd", C, D, int(width), int(height),
                      int(tile_size), tw, th, _ptr(means2d), _ptr(ray_transforms), _ptr(colors),
                      _ptr(depths), _ptr(opacities), _ptr(normals), _ptr(backgrounds),
                      _ptr(masks_u8),
                      _ptr(isect_offsets), flatten_ids.numel(), _ptr(n_dev), _ptr(flatten_ids),
                      _ptr(records), _ptr(order), _ptr(render_colors), _ptr(render_alphas), _ptr(render_normals),
                      _ptr(render_distort), _ptr(render_median), _ptr(last_ids),
                      _ptr(median_ids), _stream())
        ctx.save_for_backward(means2d, ray_transforms, colors, opacities, normals, densify,
                              backgrounds, masks_u8, isect_offsets, flatten_ids, render_colors,
                              render_alphas, last_ids, median_ids, depths)
        ctx.width, ctx.height, ctx.tile_size = int(width), int(height), int(tile_size)
        ctx.absgrad, ctx.distloss = absgrad, distloss
        ctx.n_dev = n_dev
        ctx.order = order
        ctx.visible = visible
        # outputs without a loss term (alphas, normals, distortion, median in
        # the trainer's RGB loss): None in the backward, not zero-filled images
        ctx.set_materialize_grads(False)
        return render_colors, render_alphas, render_normals, render_distort, render_median

    @staticmethod
    def backward(ctx, v_render_colors, v_render_alphas, v_render_normals, v_render_distort,
                 v_render_median):
        (means2d, ray_transforms, colors, opacities, normals, densify, backgrounds, masks_u8,
         isect_offsets, flatten_ids, render_colors, render_alphas, last_ids,
         median_ids, depths) = ctx.saved_tensors
        C, th, tw = isect_offsets.shape
        D = colors.shape[-1] + (1 if depths is not None else 0)
        H, W = ctx.height, ctx.width
        dev = means2d.device

        def grad(t, shape):
            return torch.zeros(shape, device=dev) if t is None else _f32c(t)

        v_render_colors = grad(v_render_colors, (C, H, W, D))
        v_render_alphas = None if v_render_alphas is None else _f32c(v_render_alphas)
        v_render_normals = None if v_render_normals is None else _f32c(v_render_normals)
        v_render_distort = None if v_render_distort is None else _f32c(v_render_distort)
        v_render_median = None if v_render_median is None else _f32c(v_render_median)
        G = opacities.numel()
        v_means2d = torch.empty_like(means2d)
        v_ray_transforms = torch.empty_like(ray_transforms)
        v_colors = torch.empty_like(colors)
        v_depths = None if depths is None else torch.empty_like(depths)
        v_opacities = torch.empty_like(opacities)
        # without a gradient of the normal image the normals' gradient is
        # exactly zero: None (the kernel skips it) instead of a zero-filled [G,3]
        v_normals = None if v_render_normals is None else torch.empty_like(normals)
        v_densify = torch.empty(densify.shape, device=dev)
        v_abs = torch.empty_like(means2d) if ctx.absgrad else None
        ws = torch.empty(max(int(_lib.query("gsplat_hip_rasterize_2dgs_bwd_workspace_bytes", G, D,
                                            int(ctx.absgrad))), 4), dtype=torch.uint8, device=dev)
        with _Timed("rasterize_2dgs_bwd"):
            _lib.call("gsplat_hip_rasterize_2dgs_bwd", C, D, W, H, ctx.tile_size, tw, th, G,
                      _ptr(means2d), _ptr(ray_transforms), _ptr(colors), _ptr(depths),
                      _ptr(opacities), _ptr(normals), _ptr(backgrounds), _ptr(masks_u8),
                      _ptr(isect_offsets),
                      flatten_ids.numel(), _ptr(ctx.n_dev), _ptr(flatten_ids), _ptr(ctx.order),
                      _ptr(ctx.visible), _ptr(render_colors),
                      _ptr(render_alphas), _ptr(last_ids), _ptr(median_ids),
                      _ptr(v_render_colors), _ptr(v_render_alphas), _ptr(v_render_normals),
                      _ptr(v_render_distort), _ptr(v_render_median), _ptr(v_means2d),
                      _ptr(v_ray_transforms), _ptr(v_colors), _ptr(v_depths), _ptr(v_opacities),
                      _ptr(v_normals),
                      _ptr(v_densify), _ptr(v_abs), _ptr(ws), ws.numel(), _stream())
        if ctx.absgrad:
            means2d.absgrad = v_abs
        v_backgrounds = None
        if ctx.needs_input_grad[6]:  # _wrapper.py:1953-1958
            v_backgrounds = (v_render_colors * (1.0 - render_alphas).float()).sum(dim=(1, 2))
        return (v_means2d, v_ray_transforms, v_colors, v_opacities, v_normals, v_densify,
                v_backgrounds, None, None, None, None, None, None, None, None, None, None, None,
                v_depths)


def rasterize_to_pixels_2dgs(
    means2d: Tensor,  # [C, N, 2]
    ray_transforms: Tensor,  # [C, N, 3, 3]
    colors: Tensor,  # [C, N, channels]
    opacities: Tensor,  # [C, N]
    normals: Tensor,  # [C, N, 3]
    densify: Tensor,  # [C, N, 2]
    image_width: int,
    image_height: int,
    tile_size: int,
    isect_offsets: Tensor,  # [C, tile_height, tile_width]
    flatten_ids: Tensor,  # [n_isects]
    backgrounds: Optional[Tensor] = None,  # [C, channels]
    masks: Optional[Tensor] = None,  # [C, tile_height, tile_width]
    packed: bool = False,
    absgrad: bool = False,
    distloss: bool = False,
    _n_isects_device: Optional[Tensor] = None,
    _visible: Optional[Tensor] = None,
    _colors_only: bool = False,
    _depths: Optional[Tensor] = None,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Rasterizes surfels to pixels (gsplat/cuda/_wrapper.py:1595-1726).

    Returns render_colors [C,H,W,channels], render_alphas [C,H,W,1],
    render_normals [C,H,W,3], render_distort [C,H,W,1], render_median
    [C,H,W,1].  The depth used by the distortion and median terms is the last
    colour channel, as in the reference.  `_n_isects_device` (private): the
    isect count on the device when flatten_ids is a capacity-sized array
    (the sync-free isect of a captured training step).  `_visible`
    (private): i32 per row of means2d, > 0 for the rows an isect references
    (the isect's tiles_per_gauss): only those get a record and a zeroed
    gradient row.  `_colors_only` (private, the training step): where the
    record path runs, render_normals / render_distort / render_median come
    back None (not formed).  `_depths` (private, [C, N]): the last colour
    channel read from it in place, `colors` holding the others (an RGB+D
    render without the concatenated copy; its gradient flows to _depths)."""
    C = isect_offsets.size(0)
    if _depths is not None:
        assert not packed and colors.shape[-1] + 1 in _SUPPORTED_D and backgrounds is None, \
            "_depths: dense, no backgrounds, a compiled channel count"
        assert _depths.shape == colors.shape[:-1], (_depths.shape, colors.shape)
    device = means2d.device
    if packed:  # flatten_ids index the [nnz] rows directly (_wrapper.py:1628-1636)
        nnz = means2d.size(0)
        assert means2d.shape == (nnz, 2), means2d.shape
        assert ray_transforms.shape == (nnz, 3, 3), ray_transforms.shape
        assert colors.shape[0] == nnz, colors.shape
        assert opacities.shape == (nnz,), opacities.shape
    else:
        N = means2d.size(1)
        assert means2d.shape == (C, N, 2), means2d.shape
        assert ray_transforms.shape == (C, N, 3, 3), ray_transforms.shape
        assert colors.shape[:2] == (C, N), colors.shape
        assert opacities.shape == (C, N), opacities.shape
    if backgrounds is not None:
        assert backgrounds.shape == (C, colors.shape[-1]), backgrounds.shape
        backgrounds = backgrounds.contiguous()

    channels = colors.shape[-1] + (1 if _depths is not None else 0)
    if channels > 512 or channels == 0:
        raise ValueError(f"Unsupported number of color channels: {channels}")
    if channels not in _SUPPORTED_D:
        # pad with zero channels before the last one so the depth stays last
        # (the reference pads with uninitialised channels, _wrapper.py:1657-1683)
        target = next((d for d in _SUPPORTED_D if d >= channels), None)
        if target is None:
            raise ValueError(f"Unsupported number of color channels: {channels} "
                             f"(this backend compiles {_SUPPORTED_D})")
        padded_channels = target - channels
        colors = torch.cat([colors[..., :-1],
                            torch.zeros(*colors.shape[:-1], padded_channels, device=device),
                            colors[..., -1:]], dim=-1)
        if backgrounds is not None:  # appended at the end, as the reference does
            backgrounds = torch.cat([backgrounds,
                                     torch.zeros(*backgrounds.shape[:-1], padded_channels,
                                                 device=device)], dim=-1)
    else:
        padded_channels = 0

    tile_height, tile_width = isect_offsets.shape[1:3]
    assert tile_height * tile_size >= image_height, \
        f"Assert Failed: {tile_height} * {tile_size} >= {image_height}"
    assert tile_width * tile_size >= image_width, \
        f"Assert Failed: {tile_width} * {tile_size} >= {image_width}"

    render_colors, render_alphas, render_normals, render_distort, render_median = \
        _RasterizeToPixels2DGS.apply(
            means2d.contiguous(), ray_transforms.contiguous(), colors.contiguous(),
            opacities.contiguous(), normals.contiguous(), densify.contiguous(), backgrounds,
            masks, image_width, image_height, tile_size, isect_offsets.contiguous(),
            flatten_ids.contiguous(), absgrad, distloss, _n_isects_device,
            None if _visible is None else _visible.to(torch.int32).contiguous().view(-1),
            _colors_only, None if _depths is None else _depths.contiguous())
    if padded_channels > 0:
        render_colors = torch.cat([render_colors[..., : -padded_channels - 1],
                                   render_colors[..., -1:]], dim=-1)
    return render_colors, render_alphas, render_normals, render_distort, render_median
