"""Per-pixel contributor lists and the torch compositing playground built on
them, backed by libgsplat_hip.so (csrc/indices.hip):

    rasterize_to_indices_in_range       gsplat/cuda/_wrapper.py:576-650
    rasterize_to_indices_in_range_2dgs  gsplat/cuda/_wrapper.py:1728-1800
    accumulate / accumulate_2dgs        gsplat/cuda/_torch_impl.py:432-516,
                                        gsplat/cuda/_torch_impl_2dgs.py:78-163
    _rasterize_to_pixels{,_2dgs}        gsplat/cuda/_torch_impl.py:519-611,
                                        gsplat/cuda/_torch_impl_2dgs.py:166-262

The index functions follow the reference's two-pass driver
(gsplat/cuda/csrc/Rasterization.cpp:224-296): a count kernel, an exclusive
scan of the per-pixel counts on the stream, one host sync for the total M,
then a write kernel.  `accumulate*` replace nerfacc's
render_weight_from_alpha / accumulate_along_rays (not installed here) with a
segmented exclusive product in torch, so they stay differentiable by
autograd exactly as in the reference.
"""

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._wrapper import _dev_check, _f32c, _ptr, _stream


def _indices(kind: int, range_start: int, range_end: int, transmittances: Tensor,
             means2d: Tensor, shape: Tensor, opacities: Tensor, image_width: int,
             image_height: int, tile_size: int, isect_offsets: Tensor,
             flatten_ids: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    C, N = means2d.shape[:2]
    assert opacities.shape == (C, N), opacities.shape
    assert isect_offsets.shape[0] == C, isect_offsets.shape
    tile_height, tile_width = isect_offsets.shape[1:3]
    assert tile_height * tile_size >= image_height, \
        f"Assert Failed: {tile_height} * {tile_size} >= {image_height}"
    assert tile_width * tile_size >= image_width, \
        f"Assert Failed: {tile_width} * {tile_size} >= {image_width}"
    assert transmittances.shape == (C, image_height, image_width), transmittances.shape
    _dev_check(transmittances, means2d, shape, opacities, isect_offsets, flatten_ids)
    dev = means2d.device
    trans = _f32c(transmittances)
    means2d, shape, opacities = _f32c(means2d), _f32c(shape), _f32c(opacities)
    offsets = isect_offsets.to(torch.int32).contiguous()
    fids = flatten_ids.to(torch.int32).contiguous()
    n_isects = fids.numel()
    rs, re = int(max(0, min(int(range_start), 2**31 - 1))), int(max(0, min(int(range_end), 2**31 - 1)))
    common = (kind, C, N, image_width, image_height, tile_size, tile_width, tile_height,
              n_isects, rs, re, _ptr(trans), _ptr(means2d), _ptr(shape), _ptr(opacities),
              _ptr(offsets), _ptr(fids))
    HW = image_width * image_height
    if n_isects == 0:
        e = torch.empty(0, dtype=torch.int64, device=dev)
        return e, e.clone(), e.clone()
    cnts = torch.empty(C * HW, dtype=torch.int32, device=dev)
    _lib.call("gsplat_hip_rasterize_to_indices_count", *common, _ptr(cnts), _stream())
    csum = torch.cumsum(cnts, 0, dtype=torch.int32)
    M = int(csum[-1].item())  # the one host sync (Rasterization.cpp:268)
    gauss_ids = torch.empty(M, dtype=torch.int64, device=dev)
    indices = torch.empty(M, dtype=torch.int64, device=dev)
    if M:
        starts = csum - cnts
        _lib.call("gsplat_hip_rasterize_to_indices_write", *common, _ptr(starts),
                  _ptr(gauss_ids), _ptr(indices), _stream())
    return gauss_ids, indices % HW, indices // HW


@torch.no_grad()
def rasterize_to_indices_in_range(range_start: int, range_end: int, transmittances: Tensor,
                                  means2d: Tensor, conics: Tensor, opacities: Tensor,
                                  image_width: int, image_height: int, tile_size: int,
                                  isect_offsets: Tensor, flatten_ids: Tensor
                                  ) -> Tuple[Tensor, Tensor, Tensor]:
    """(gaussian_ids, pixel_ids, camera_ids), each int64 [M]: every (Gaussian,
    pixel) pair that contributes to the composite when the tiles' depth-sorted
    lists are walked over batches [range_start, range_end) of tile_size**2
    records, starting from `transmittances` [C, H, W]
    (gsplat/cuda/_wrapper.py:576-650).  Pixel-major, front-to-back order."""
    C, N = means2d.shape[:2]
    assert conics.shape == (C, N, 3), conics.shape
    return _indices(0, range_start, range_end, transmittances, means2d, conics, opacities,
                    image_width, image_height, tile_size, isect_offsets, flatten_ids)


@torch.no_grad()
def rasterize_to_indices_in_range_2dgs(range_start: int, range_end: int,
                                       transmittances: Tensor, means2d: Tensor,
                                       ray_transforms: Tensor, opacities: Tensor,
                                       image_width: int, image_height: int, tile_size: int,
                                       isect_offsets: Tensor, flatten_ids: Tensor
                                       ) -> Tuple[Tensor, Tensor, Tensor]:
    """2DGS counterpart of `rasterize_to_indices_in_range`
    (gsplat/cuda/_wrapper.py:1728-1800): the surfel weight is
    min(|s(ray)|^2, 2 |p - mean2d|^2) as in RasterizeToIndices2DGS.cu:150-176."""
    C, N = means2d.shape[:2]
    assert ray_transforms.shape == (C, N, 3, 3), ray_transforms.shape
    return _indices(1, range_start, range_end, transmittances, means2d, ray_transforms,
                    opacities, image_width, image_height, tile_size, isect_offsets, flatten_ids)


# ------------------------------------------------ torch compositing playground

def _render_weights(alphas: Tensor, ray_ids: Tensor) -> Tensor:
    """alpha_i * prod_{j < i, same ray} (1 - alpha_j) for entries grouped by ray
    in front-to-back order (nerfacc.render_weight_from_alpha's packed case)."""
    if alphas.numel() == 0:
        return alphas
    lt = torch.log1p(-alphas.double())
    cs = torch.cumsum(lt, 0)
    excl = cs - lt
    first = torch.ones_like(ray_ids, dtype=torch.bool)
    first[1:] = ray_ids[1:] != ray_ids[:-1]
    seg = torch.cumsum(first.long(), 0) - 1
    base = excl[first][seg]
    return (alphas.double() * torch.exp(excl - base)).to(alphas.dtype)


def _along_rays(weights: Tensor, values: Optional[Tensor], ray_ids: Tensor, n_rays: int) -> Tensor:
    src = weights[:, None] if values is None else weights[:, None] * values
    out = torch.zeros((n_rays, src.shape[-1]), dtype=src.dtype, device=src.device)
    return out.index_add(0, ray_ids, src)


def accumulate(means2d: Tensor, conics: Tensor, opacities: Tensor, colors: Tensor,
               gaussian_ids: Tensor, pixel_ids: Tensor, camera_ids: Tensor,
               image_width: int, image_height: int) -> Tuple[Tensor, Tensor]:
    """Alpha compositing of the given (Gaussian, pixel, camera) triples in
    plain torch, differentiable by autograd (gsplat/cuda/_torch_impl.py:432-516).
    The triples must be grouped by pixel, front to back (the order
    `rasterize_to_indices_in_range` returns)."""
    C = means2d.shape[0]
    channels = colors.shape[-1]
    px = pixel_ids % image_width
    py = pixel_ids // image_width
    coords = torch.stack([px, py], -1) + 0.5
    deltas = coords - means2d[camera_ids, gaussian_ids]
    c = conics[camera_ids, gaussian_ids]
    sigmas = 0.5 * (c[:, 0] * deltas[:, 0] ** 2 + c[:, 2] * deltas[:, 1] ** 2) \
        + c[:, 1] * deltas[:, 0] * deltas[:, 1]
    alphas = torch.clamp_max(opacities[camera_ids, gaussian_ids] * torch.exp(-sigmas), 0.999)
    rays = camera_ids * image_height * image_width + pixel_ids
    n_rays = C * image_height * image_width
    w = _render_weights(alphas, rays)
    renders = _along_rays(w, colors[camera_ids, gaussian_ids], rays, n_rays)
    accs = _along_rays(w, None, rays, n_rays)
    return (renders.reshape(C, image_height, image_width, channels),
            accs.reshape(C, image_height, image_width, 1))


def accumulate_2dgs(means2d: Tensor, ray_transforms: Tensor, opacities: Tensor, colors: Tensor,
                    normals: Tensor, gaussian_ids: Tensor, pixel_ids: Tensor,
                    camera_ids: Tensor, image_width: int, image_height: int
                    ) -> Tuple[Tensor, Tensor, Tensor]:
    """2DGS compositing of contributor triples in plain torch
    (gsplat/cuda/_torch_impl_2dgs.py:78-163): renders, alphas, normals."""
    C = means2d.shape[0]
    channels = colors.shape[-1]
    px = pixel_ids % image_width + 0.5
    py = pixel_ids // image_width + 0.5
    deltas = torch.stack([px, py], -1) - means2d[camera_ids, gaussian_ids]
    M = ray_transforms[camera_ids, gaussian_ids]
    h_u = -M[..., 0, :] + M[..., 2, :] * px[..., None]
    h_v = -M[..., 1, :] + M[..., 2, :] * py[..., None]
    t = torch.cross(h_u, h_v, dim=-1)
    us, vs = t[..., 0] / t[..., 2], t[..., 1] / t[..., 2]
    sig = 0.5 * torch.minimum(us ** 2 + vs ** 2, 2 * (deltas[..., 0] ** 2 + deltas[..., 1] ** 2))
    alphas = torch.clamp_max(opacities[camera_ids, gaussian_ids] * torch.exp(-sig), 0.999)
    rays = camera_ids * image_height * image_width + pixel_ids
    n_rays = C * image_height * image_width
    w = _render_weights(alphas, rays)
    shp = (C, image_height, image_width)
    return (_along_rays(w, colors[camera_ids, gaussian_ids], rays, n_rays).reshape(*shp, channels),
            _along_rays(w, None, rays, n_rays).reshape(*shp, 1),
            _along_rays(w, normals[camera_ids, gaussian_ids], rays, n_rays).reshape(*shp, 3))


def _num_batches(isect_offsets: Tensor, n_isects: int, tile_size: int) -> int:
    fl = torch.cat([isect_offsets.flatten().long(),
                    torch.tensor([n_isects], device=isect_offsets.device)])
    max_range = int((fl[1:] - fl[:-1]).max().item())
    bs = tile_size * tile_size
    return (max_range + bs - 1) // bs


def _rasterize_to_pixels(means2d: Tensor, conics: Tensor, colors: Tensor, opacities: Tensor,
                         image_width: int, image_height: int, tile_size: int,
                         isect_offsets: Tensor, flatten_ids: Tensor,
                         backgrounds: Optional[Tensor] = None, batch_per_iter: int = 100):
    """Iterative rasterization through the index lists and `accumulate`
    (gsplat/cuda/_torch_impl.py:519-611); differentiable by autograd."""
    C = means2d.shape[0]
    dev = means2d.device
    rc = torch.zeros((C, image_height, image_width, colors.shape[-1]), device=dev)
    ra = torch.zeros((C, image_height, image_width, 1), device=dev)
    nb = _num_batches(isect_offsets, len(flatten_ids), tile_size)
    for step in range(0, nb, batch_per_iter):
        trans = 1.0 - ra[..., 0]
        gs, pix, cam = rasterize_to_indices_in_range(
            step, step + batch_per_iter, trans.detach(), means2d.detach(), conics.detach(),
            opacities.detach(), image_width, image_height, tile_size, isect_offsets, flatten_ids)
        if len(gs) == 0:
            break
        r, a = accumulate(means2d, conics, opacities, colors, gs, pix, cam,
                          image_width, image_height)
        rc = rc + r * trans[..., None]
        ra = ra + a * trans[..., None]
    if backgrounds is not None:
        rc = rc + backgrounds[:, None, None, :] * (1.0 - ra)
    return rc, ra


def _rasterize_to_pixels_2dgs(means2d: Tensor, ray_transforms: Tensor, colors: Tensor,
                              normals: Tensor, opacities: Tensor, image_width: int,
                              image_height: int, tile_size: int, isect_offsets: Tensor,
                              flatten_ids: Tensor, backgrounds: Optional[Tensor] = None,
                              batch_per_iter: int = 100):
    """2DGS iterative rasterization through the index lists
    (gsplat/cuda/_torch_impl_2dgs.py:166-262)."""
    C = means2d.shape[0]
    dev = means2d.device
    rc = torch.zeros((C, image_height, image_width, colors.shape[-1]), device=dev)
    ra = torch.zeros((C, image_height, image_width, 1), device=dev)
    rn = torch.zeros((C, image_height, image_width, 3), device=dev)
    nb = _num_batches(isect_offsets, len(flatten_ids), tile_size)
    for step in range(0, nb, batch_per_iter):
        trans = 1.0 - ra[..., 0]
        gs, pix, cam = rasterize_to_indices_in_range_2dgs(
            step, step + batch_per_iter, trans.detach(), means2d.detach(),
            ray_transforms.detach(), opacities.detach(), image_width, image_height, tile_size,
            isect_offsets, flatten_ids)
        if len(gs) == 0:
            break
        r, a, n = accumulate_2dgs(means2d, ray_transforms, opacities, colors, normals, gs, pix,
                                  cam, image_width, image_height)
        rc = rc + r * trans[..., None]
        ra = ra + a * trans[..., None]
        rn = rn + n * trans[..., None]
    if backgrounds is not None:
        rc = rc + backgrounds[:, None, None, :] * (1.0 - ra)
    return rc, ra, rn
