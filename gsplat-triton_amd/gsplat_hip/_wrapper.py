"""The 5-function backend surface of gsplat, backed by libgsplat_hip.so.

Drop-in for `gsplat/triton_impl/_wrapper.py` (the functions that
`gsplat/rendering.py:11-29` imports from the selected backend):

    fully_fused_projection   _wrapper.py:429-541  (autograd: _FullyFusedProjection :300)
    isect_tiles              _wrapper.py:544 -> isect_tiles.py:13-131   (no grad)
    isect_offset_encode      _wrapper.py:548 -> isect_offset.py:8-33    (no grad)
    spherical_harmonics      _wrapper.py:596-620  (autograd: _SphericalHarmonics :552)
    rasterize_to_pixels      _wrapper.py:185-297  (autograd: _RasterizeToPixels :42)

Same signatures, defaults, assertions, error types and autograd contract
(argument order, `None` gradients, `ctx.needs_input_grad[4]` gating,
`means2d.absgrad`).  Every op runs through the HIP C ABI on torch's current
stream; there is no CPU or Triton fallback.
"""

import contextlib
import ctypes
import math
import os
import time
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib

_SUPPORTED_D = (1, 2, 3, 4, 8, 16, 32)


def _ptr(t: Optional[Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream() -> int:
    """torch's current HIP stream on the current device, as a raw handle
    (the C accessors: torch.cuda.current_stream() builds a Stream object,
    ~10 us of host time per launch on a slow host)."""
    if _raw_stream is not None and _cur_device is not None:
        return _raw_stream(_cur_device())
    return torch.cuda.current_stream().cuda_stream


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.GsplatHipError(
                "gsplat_hip ops run on the GPU only; got a tensor on " + str(t.device))


def _f32c(t: Optional[Tensor]) -> Optional[Tensor]:
    if t is None:
        return None
    return t.contiguous() if t.dtype == torch.float32 else t.float().contiguous()


def _aligned16(t: Tensor) -> Tensor:
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _bit_length(x: int) -> int:
    return int(x).bit_length()


# Optional per-kernel timing (bench.py): when enabled, HIP events are recorded
# on the launch stream immediately around the named C-ABI calls.
_timers = None


def enable_kernel_timers(enabled: bool = True):
    global _timers
    _timers = {} if enabled else None
    return _timers


class _Timed:
    __slots__ = ("name", "ev")

    def __init__(self, name):
        self.name = name
        self.ev = None

    def __enter__(self):
        if _timers is not None:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record()
        return self

    def __exit__(self, *exc):
        if self.ev is not None:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            _timers.setdefault(self.name, []).append((self.ev, end))
        return False


# ============================================================== projection ==
class _FullyFusedProjection(torch.autograd.Function):
    """Projects Gaussians to 2D (gsplat/triton_impl/_wrapper.py:300-426)."""

    @staticmethod
    def forward(ctx, means, covars, quats, scales, viewmats, Ks, width, height, eps2d,
                near_plane, far_plane, radius_clip, calc_compensations,
                camera_model="pinhole", block_size=256, fusion=None):
        if camera_model != "pinhole":
            raise NotImplementedError(f"Unsupported camera model: {camera_model}")
        ctx.set_materialize_grads(False)  # unused outputs: None, no zero-filled buffers
        ctx.fusion = fusion  # a training step's StepFusion (geometry Adam in this backward)
        assert (covars is None) and (quats is not None) and (scales is not None)
        means, quats, scales, viewmats, Ks = (_f32c(x) for x in (means, quats, scales, viewmats, Ks))
        quats = _aligned16(quats)
        _dev_check(means, quats, scales, viewmats, Ks)
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device
        radii = torch.empty((C, N), dtype=torch.int32, device=dev)
        means2d = torch.empty((C, N, 2), dtype=torch.float32, device=dev)
        depths = torch.empty((C, N), dtype=torch.float32, device=dev)
        conics = torch.empty((C, N, 3), dtype=torch.float32, device=dev)
        comps = torch.empty((C, N), dtype=torch.float32, device=dev) if calc_compensations else None
        _lib.call("gsplat_hip_projection_fwd", C, N, _ptr(means), _ptr(quats), _ptr(scales),
                  _ptr(viewmats), _ptr(Ks), int(width), int(height), float(eps2d),
                  float(near_plane), float(far_plane), float(radius_clip), _ptr(radii),
                  _ptr(means2d), _ptr(depths), _ptr(conics), _ptr(comps), _stream())
        ctx.save_for_backward(means, quats, scales, viewmats, Ks, radii, conics, comps)
        ctx.width, ctx.height, ctx.eps2d = int(width), int(height), float(eps2d)
        ctx.mark_non_differentiable(radii)
        return radii, means2d, depths, conics, comps

    @staticmethod
    def backward(ctx, v_radii, v_means2d, v_depths, v_conics, v_compensations):
        means, quats, scales, viewmats, Ks, radii, conics, comps = ctx.saved_tensors
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device

        def g(t, shape):
            return torch.zeros(shape, device=dev) if t is None else _f32c(t)

        v_means2d = g(v_means2d, (C, N, 2))
        v_depths = None if v_depths is None else _f32c(v_depths)  # null = zeros in the kernel
        v_conics = g(v_conics, (C, N, 3))
        if comps is not None:
            v_compensations = g(v_compensations, (C, N))
        else:
            v_compensations = None
        want_vm = ctx.needs_input_grad[4]
        fusion = ctx.fusion
        if (fusion is not None and C == 1 and comps is None and not want_vm
                and fusion.geom_adam_ready()):
            # the trainer's geometry Adam step in this backward: no gradients
            # stored (gsplat_hip_projection_bwd_adam)
            fusion.geom_adam.run(means, quats, scales, viewmats, Ks, ctx.width, ctx.height,
                                 ctx.eps2d, radii, conics, v_means2d, v_depths, v_conics, fusion)
            return (None,) * 16
        v_means = torch.empty((N, 3), device=dev)
        v_quats = torch.empty((N, 4), device=dev)
        v_scales = torch.empty((N, 3), device=dev)
        v_viewmats = torch.empty((C, 4, 4), device=dev) if want_vm else None
        _lib.call("gsplat_hip_projection_bwd", C, N, _ptr(means), _ptr(quats), _ptr(scales),
                  _ptr(viewmats), _ptr(Ks), ctx.width, ctx.height, ctx.eps2d, _ptr(radii),
                  _ptr(conics), _ptr(comps), _ptr(v_means2d), _ptr(v_depths), _ptr(v_conics),
                  _ptr(v_compensations), _ptr(v_means), _ptr(v_quats), _ptr(v_scales),
                  _ptr(v_viewmats), _stream())
        return (v_means if ctx.needs_input_grad[0] else None, None,
                v_quats if ctx.needs_input_grad[2] else None,
                v_scales if ctx.needs_input_grad[3] else None,
                v_viewmats, None, None, None, None, None, None, None, None, None, None, None)


class _FullyFusedProjectionPacked(torch.autograd.Function):
    """Projects Gaussians to 2D, packed [nnz] outputs
    (gsplat/cuda/_wrapper.py:998-1190; broken on the Triton backend).
    One host read of nnz, as the reference's cumsum(...)[-1].item()."""

    @staticmethod
    def forward(ctx, means, covars, quats, scales, viewmats, Ks, width, height, eps2d,
                near_plane, far_plane, radius_clip, sparse_grad, calc_compensations,
                camera_model="pinhole"):
        if camera_model != "pinhole":
            raise NotImplementedError(f"Unsupported camera model: {camera_model}")
        assert covars is None and quats is not None and scales is not None
        means, quats, scales, viewmats, Ks = (_f32c(x) for x in (means, quats, scales, viewmats, Ks))
        quats = _aligned16(quats)
        _dev_check(means, quats, scales, viewmats, Ks)
        C, N = viewmats.shape[0], means.shape[0]
        dev = means.device
        ws = torch.empty(max(int(_lib.query("gsplat_hip_projection_packed_workspace_bytes", C, N))
                             // 8, 1), dtype=torch.int64, device=dev)
        nnz_dev = torch.empty(1, dtype=torch.int64, device=dev)
        args = (_ptr(means), _ptr(quats), _ptr(scales), _ptr(viewmats), _ptr(Ks), int(width),
                int(height), float(eps2d), float(near_plane), float(far_plane), float(radius_clip))
        _lib.call("gsplat_hip_projection_packed_count", C, N, *args, _ptr(ws), _ptr(nnz_dev),
                  _stream())
        nnz = int(nnz_dev.item())
        camera_ids = torch.empty(nnz, dtype=torch.int64, device=dev)
        gaussian_ids = torch.empty(nnz, dtype=torch.int64, device=dev)
        radii = torch.empty(nnz, dtype=torch.int32, device=dev)
        means2d = torch.empty((nnz, 2), device=dev)
        depths = torch.empty(nnz, device=dev)
        conics = torch.empty((nnz, 3), device=dev)
        comps = torch.empty(nnz, device=dev) if calc_compensations else None
        _lib.call("gsplat_hip_projection_packed_fwd", C, N, *args, _ptr(ws), _ptr(camera_ids),
                  _ptr(gaussian_ids), _ptr(radii), _ptr(means2d), _ptr(depths), _ptr(conics),
                  _ptr(comps), _stream())
        ctx.save_for_backward(camera_ids, gaussian_ids, means, quats, scales, viewmats, Ks,
                              conics, comps)
        ctx.width, ctx.height, ctx.eps2d = int(width), int(height), float(eps2d)
        ctx.sparse_grad = sparse_grad
        ctx.mark_non_differentiable(camera_ids, gaussian_ids, radii)
        return camera_ids, gaussian_ids, radii, means2d, depths, conics, comps

    @staticmethod
    def backward(ctx, v_camera_ids, v_gaussian_ids, v_radii, v_means2d, v_depths, v_conics,
                 v_compensations):
        camera_ids, gaussian_ids, means, quats, scales, viewmats, Ks, conics, comps = \
            ctx.saved_tensors
        C, N, nnz = viewmats.shape[0], means.shape[0], camera_ids.numel()
        dev = means.device

        def g(t, shape):
            return torch.zeros(shape, device=dev) if t is None else _f32c(t)

        v_means2d = g(v_means2d, (nnz, 2))
        v_conics = g(v_conics, (nnz, 3))
        v_depths = None if v_depths is None else _f32c(v_depths)
        v_comps = g(v_compensations, (nnz,)) if comps is not None else None
        rows = nnz if ctx.sparse_grad else N
        v_means = torch.empty((rows, 3), device=dev)
        v_quats = torch.empty((rows, 4), device=dev)
        v_scales = torch.empty((rows, 3), device=dev)
        v_viewmats = torch.empty((C, 4, 4), device=dev) if ctx.needs_input_grad[4] else None
        _lib.call("gsplat_hip_projection_packed_bwd", C, N, nnz, _ptr(means), _ptr(quats),
                  _ptr(scales), _ptr(viewmats), _ptr(Ks), ctx.width, ctx.height, ctx.eps2d,
                  _ptr(camera_ids), _ptr(gaussian_ids), _ptr(conics), _ptr(comps),
                  _ptr(v_means2d), _ptr(v_depths), _ptr(v_conics), _ptr(v_comps),
                  int(bool(ctx.sparse_grad)), _ptr(v_means), _ptr(v_quats), _ptr(v_scales),
                  _ptr(v_viewmats), _stream())
        if ctx.sparse_grad:  # COO gradients (_wrapper.py:1127-1170)
            def coo(v, like):
                return torch.sparse_coo_tensor(indices=gaussian_ids[None], values=v,
                                               size=like.size(), is_coalesced=C == 1)
            v_means, v_quats, v_scales = coo(v_means, means), coo(v_quats, quats), \
                coo(v_scales, scales)
        return (v_means if ctx.needs_input_grad[0] else None, None,
                v_quats if ctx.needs_input_grad[2] else None,
                v_scales if ctx.needs_input_grad[3] else None,
                v_viewmats, None, None, None, None, None, None, None, None, None, None)


def fully_fused_projection(
    means: Tensor,  # [N, 3]
    covars: Optional[Tensor],  # must be None (quats/scales path only, as the Triton backend)
    quats: Optional[Tensor],  # [N, 4]
    scales: Optional[Tensor],  # [N, 3]
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
    calc_compensations: bool = False,
    camera_model: str = "pinhole",
    block_size: int = 256,
) -> Tuple[Tensor, Tensor, Tensor, Tensor, Optional[Tensor]]:
    """Projects Gaussians to 2D (gsplat/triton_impl/_wrapper.py:429-541).

    Returns radii i32[C,N], means2d [C,N,2], depths [C,N], conics [C,N,3],
    compensations [C,N] or None.  Entries with radii == 0 are invalid (written
    as zeros here; the reference leaves them uninitialised).  packed=True
    returns (camera_ids, gaussian_ids, radii, means2d, depths, conics,
    compensations) over the nnz kept pairs, as the CUDA backend
    (gsplat/cuda/_wrapper.py:998-1190); sparse_grad makes the gradients of
    means/quats/scales COO tensors."""
    C = viewmats.size(0)
    N = means.size(0)
    assert means.size() == (N, 3), means.size()
    assert viewmats.size() == (C, 4, 4), viewmats.size()
    assert Ks.size() == (C, 3, 3), Ks.size()
    assert covars is None
    assert quats is not None, "covars or quats is required"
    assert scales is not None, "covars or scales is required"
    assert quats.size() == (N, 4), quats.size()
    assert scales.size() == (N, 3), scales.size()
    if sparse_grad:
        assert packed, "sparse_grad is only supported when packed is True"
    if packed:
        return _FullyFusedProjectionPacked.apply(
            means.contiguous(), covars, quats.contiguous(), scales.contiguous(),
            viewmats.contiguous(), Ks.contiguous(), width, height, eps2d, near_plane, far_plane,
            radius_clip, sparse_grad, calc_compensations, camera_model)
    return _FullyFusedProjection.apply(means, covars, quats, scales, viewmats, Ks, width, height,
                                       eps2d, near_plane, far_plane, radius_clip,
                                       calc_compensations, camera_model, block_size)


# =================================================================== isect ==
# Sorted-isect strategy (csrc/isect.hip), all with identical output:
#   "tile_first"  stable 32-bit (camera, tile) sort + segmented depth sort
#   "depth_first" depth sort of the visible Gaussians + stable (camera, tile) sort
#   "full"        the reference's single 64-bit key sort
ISECT_SORT = os.environ.get("GSPLAT_HIP_ISECT_SORT", "depth_first")
# 16x16 rasterizer gathers from packed 64-B render records (GSPLAT_HIP_RECORDS=0:
# from the four attribute arrays, as before ABI 15)
RECORDS = os.environ.get("GSPLAT_HIP_RECORDS", "1") != "0"
# render records and gradient rows indexed by the Gaussians' depth rank among
# the visible ones (isect supertile expansion's rank ids): the live rows are
# the first n_visible, in depth order (GSPLAT_HIP_RANKS=0: indexed by Gaussian)
RANKS = os.environ.get("GSPLAT_HIP_RANKS", "1") != "0"
# longest busy-poll of the n_isects copy before a blocking event wait (s)
SPIN_S = float(os.environ.get("GSPLAT_HIP_SYNC_SPIN_US", "2000")) * 1e-6


@torch.no_grad()
def isect_tiles(
    means2d: Tensor,  # [C, N, 2] or [nnz, 2]
    radii: Tensor,  # [C, N] or [nnz]
    depths: Tensor,  # [C, N] or [nnz]
    tile_size: int,
    tile_width: int,
    tile_height: int,
    sort: bool = True,
    packed: bool = False,
    n_cameras: Optional[int] = None,
    camera_ids: Optional[Tensor] = None,
    gaussian_ids: Optional[Tensor] = None,
    block_size: int = 256,
) -> Tuple[Tensor, Tensor, Tensor]:
    """Maps projected Gaussians to intersecting tiles (isect_tiles.py:13-131).

    Returns tiles_per_gauss i32 [C,N] (or [nnz]), isect_ids i64 [n_isects]
    (camera | tile | depth bits, Triton tile-bit width) and flatten_ids i32.
    One device->host read of n_isects, as the reference."""
    return isect_tiles_begin(means2d, radii, depths, tile_size, tile_width, tile_height, packed,
                             n_cameras, camera_ids, gaussian_ids).finish(sort)


def isect_tiles_begin(means2d, radii, depths, tile_size, tile_width, tile_height,
                      packed=False, n_cameras=None, camera_ids=None, gaussian_ids=None,
                      sync=True):
    """First half of isect_tiles (counts queued, totals on their way to the
    host); `.finish(sort)` returns isect_tiles' outputs.  sync=False: the
    totals stay on the device and `.finish_capped(capacity)` emits into
    fixed-size arrays without any host synchronisation."""
    dev = means2d.device
    if packed:
        nnz = means2d.size(0)
        assert means2d.shape == (nnz, 2), means2d.size()
        assert radii.shape == (nnz,), radii.size()
        assert depths.shape == (nnz,), depths.size()
        assert camera_ids is not None, "camera_ids is required if packed is True"
        assert gaussian_ids is not None, "gaussian_ids is required if packed is True"
        assert n_cameras is not None, "n_cameras is required if packed is True"
        C, N, G = n_cameras, 0, nnz
        camera_ids = camera_ids.to(torch.int32).contiguous()
    else:
        C, N, _ = means2d.shape
        G = C * N
        assert means2d.shape == (C, N, 2), means2d.size()
        assert radii.shape == (C, N), radii.size()
        assert depths.shape == (C, N), depths.size()
        camera_ids = None
    means2d = _f32c(means2d)
    radii = radii.to(torch.int32).contiguous()
    depths = _f32c(depths)
    _dev_check(means2d, radii, depths)
    n_bit_tile = _bit_length(tile_height * tile_width - 1)
    n_bit_cam = _bit_length(C - 1)
    assert n_bit_tile + n_bit_cam <= 32, "tile_id and cam_id exceed 32 bits"

    return _IsectCount(means2d, radii, depths, camera_ids, C, N, G, tile_size, tile_width,
                       tile_height, n_bit_tile, n_bit_cam, packed, sync)


class _IsectCount:
    """isect_tiles in two halves around its single host sync: the count
    kernels and an asynchronous copy of (n_isects, n_visible) into pinned host
    memory are queued on construction; `finish` waits for that copy only and
    queues the emission and sort.  Work queued in between (rasterization()'s
    SH colours) keeps the GPU busy across the host round trip."""

    def __init__(self, means2d, radii, depths, camera_ids, C, N, G, tile_size, tile_width,
                 tile_height, n_bit_tile, n_bit_cam, packed, sync=True):
        dev = means2d.device
        self.args = (means2d, radii, depths, camera_ids, C, N, G, tile_size, tile_width,
                     tile_height, n_bit_tile, n_bit_cam, packed)
        self.tpg = torch.empty(G, dtype=torch.int32, device=dev)
        self.offsets = None  # the tile offsets, when the emission produced them
        # (rank_ids [n_isects], vis_rank [G]) when the emission produced them
        self.ranks = None
        self.ws = torch.empty(max(int(_lib.query("gsplat_hip_isect_workspace_bytes", G)), 8),
                              dtype=torch.uint8, device=dev)
        totals = torch.empty(2, dtype=torch.int64, device=dev)
        _lib.call("gsplat_hip_isect_count", G, _ptr(means2d), _ptr(radii), tile_size,
                  tile_width, tile_height, _ptr(self.tpg), _ptr(self.ws), _ptr(totals),
                  _stream())
        self.totals = totals
        if not sync:
            self.host = self.event = None
            return
        # a pinned buffer of its own per call (torch's caching host allocator
        # recycles it only after the copy's event): concurrent begins on other
        # streams or threads cannot overwrite each other's totals
        host = torch.empty(2, dtype=torch.int64, pin_memory=True)
        host.copy_(totals, non_blocking=True)
        self.host, self.totals = host, totals
        self.event = torch.cuda.Event(blocking=True)
        self.event.record()

    @torch.no_grad()
    def finish(self, sort: bool = True, ranks: bool = True) -> Tuple[Tensor, Tensor, Tensor]:
        (means2d, radii, depths, camera_ids, C, N, G, tile_size, tile_width, tile_height,
         n_bit_tile, n_bit_cam, packed) = self.args
        dev, st = means2d.device, _stream()
        tpg, ws = self.tpg, self.ws
        # the single host sync (isect_tiles.py:102); polling reacts within a
        # few us where hipEventSynchronize's blocking wait took ~100 us, so
        # poll for up to SPIN_S (the counts normally land well inside it),
        # then park the thread in the blocking-sync event wait instead of
        # holding a core when the stream is deep in other work
        t_end = time.perf_counter() + SPIN_S
        while not self.event.query():
            if time.perf_counter() > t_end:
                self.event.synchronize()
                break
            time.sleep(0)  # yields the core (and the GIL) between polls
        n_isects, n_visible = self.host.tolist()
        isect_ids = torch.empty(n_isects, dtype=torch.int64, device=dev)
        flatten_ids = torch.empty(n_isects, dtype=torch.int32, device=dev)
        if sort and ISECT_SORT == "tile_first" and n_isects > 0:
            sws = torch.empty(max(int(_lib.query("gsplat_hip_isect_tilefirst_workspace_bytes",
                                                 n_isects, C * tile_width * tile_height,
                                                 n_bit_tile + n_bit_cam)), 8),
                              dtype=torch.uint8, device=dev)
            _lib.call("gsplat_hip_isect_write_tilefirst", G, N, _ptr(means2d), _ptr(radii),
                      _ptr(depths), _ptr(camera_ids), tile_size, tile_width, tile_height, C,
                      n_bit_tile, n_bit_cam, _ptr(ws), n_isects, _ptr(sws), sws.numel(),
                      _ptr(isect_ids), _ptr(flatten_ids), st)
        elif sort and ISECT_SORT == "depth_first":
            key_bits = n_bit_tile + n_bit_cam
            sws = torch.empty(max(int(_lib.query("gsplat_hip_isect_sorted_workspace_bytes", n_visible,
                                                 n_isects, key_bits)), 8),
                              dtype=torch.uint8, device=dev)
            # the tile offsets come with the isects (supertile expansion,
            # csrc/isect_st.h): rasterization() reads them from `.offsets`
            self.offsets = torch.empty((C, tile_height, tile_width), dtype=torch.int32,
                                       device=dev)
            rk = self._rank_buffers(n_isects) if ranks else None
            _lib.call("gsplat_hip_isect_write_sorted", G, N, _ptr(means2d), _ptr(radii),
                      _ptr(depths), _ptr(camera_ids), _ptr(tpg), tile_size, tile_width, tile_height,
                      n_bit_tile, n_bit_cam, _ptr(ws), n_visible, n_isects, _ptr(sws), sws.numel(),
                      _ptr(isect_ids), _ptr(flatten_ids), C, _ptr(self.offsets),
                      *(_ptr(t) for t in (rk or (None, None))), st)
            self.ranks = rk
        else:
            _lib.call("gsplat_hip_isect_write", G, N, _ptr(means2d), _ptr(radii), _ptr(depths),
                      _ptr(camera_ids), tile_size, tile_width, tile_height, n_bit_tile, _ptr(ws),
                      _ptr(isect_ids), _ptr(flatten_ids), st)
            if sort and n_isects > 0:
                sws = torch.empty(max(int(_lib.query("gsplat_hip_sort_workspace_bytes", n_isects)),
                                      8), dtype=torch.uint8, device=dev)
                keys = torch.empty_like(isect_ids)
                vals = torch.empty_like(flatten_ids)
                _lib.call("gsplat_hip_radix_sort", n_isects, 32 + n_bit_tile + n_bit_cam,
                          _ptr(isect_ids), _ptr(flatten_ids), _ptr(keys), _ptr(vals), _ptr(sws),
                          sws.numel(), st)
                isect_ids, flatten_ids = keys, vals
        if not packed:
            tpg = tpg.view(C, N)
        return tpg, isect_ids, flatten_ids

    def will_rank(self, capped: bool = False) -> bool:
        """Whether finish(sort=True) / finish_capped will also return the depth
        ranks (`.ranks`): render records packed before then would be indexed
        by Gaussian, not by rank."""
        (_, _, _, _, C, _, _, _, tile_width, tile_height, _, _, packed) = self.args
        return (RANKS and not packed and (capped or ISECT_SORT == "depth_first")
                and bool(_lib.query("gsplat_hip_isect_ranked", C, tile_width, tile_height)))

    def _rank_buffers(self, n_slots, capped=False):
        """(rank_ids [n_slots], vis_rank [G]) when the sorted emission can write
        the depth ranks (supertile expansion), else None."""
        means2d, G = self.args[0], self.args[6]
        if G == 0 or not self.will_rank(capped):
            return None
        dev = means2d.device
        return (torch.empty(max(int(n_slots), 1), dtype=torch.int32, device=dev),
                torch.empty(G, dtype=torch.int32, device=dev))

    @torch.no_grad()
    def finish_capped(self, capacity: int, status: Optional[Tensor] = None, report=None,
                      ids: bool = True, ranks: bool = True, surfel_cull=None):
        """The sorted isects with NO host synchronisation (the one sync of
        isect_tiles, isect_tiles.py:101-102, removed so that a training step
        can be captured into a HIP graph): isect_ids / flatten_ids have
        `capacity` slots, of which counts[0] (device i64) are written --
        the same isects as finish(sort=True) -- or none if they do not fit
        (counts[2] = 1; status[0] |= 1, sticky, when given); counts[1] = the
        visible Gaussians, counts[3] = n_isects whether it fit or not.
        `report` = (device pointer of a host-mapped i64[ring][4], device i64
        slot tensor): the counts also go to that ring row.  ids=False (a
        caller that only walks the depth ranks, the training step; needs
        will_rank(capped=True)): isect_ids / flatten_ids are not written and
        come back None -- the rank ids and offsets are.  ranks=False: no depth
        ranks (a rasterizer that gathers by Gaussian id, the 2DGS one); with
        ids=False too (the 2DGS training step, ABI 33) only flatten_ids and
        the offsets are written, isect_ids comes back None (where the
        supertile expansion runs; else both are written).  surfel_cull =
        (ray_transforms [C,N,3,3], opacities [C,N]) with ids=False,
        ranks=False (the 2DGS training step, ABI 34): large surfels get isects
        only in the tiles their image can reach
        (gsplat_hip_isect_write_sorted_capped_surfel); counts[0] is then the
        number written, counts[3] the tile-rectangle count.  Returns
        (tiles_per_gauss, isect_ids, flatten_ids, counts)."""
        (means2d, radii, depths, camera_ids, C, N, G, tile_size, tile_width, tile_height,
         n_bit_tile, n_bit_cam, packed) = self.args
        dev = means2d.device
        capacity = int(capacity)
        key_bits = n_bit_tile + n_bit_cam
        ws = torch.empty(max(int(_lib.query("gsplat_hip_isect_sorted_capped_workspace_bytes", G,
                                            capacity, key_bits)), 8),
                         dtype=torch.uint8, device=dev)
        rk = self._rank_buffers(capacity, capped=True) if ranks else None
        flat_only = not ids and not ranks and G > 0 and self.will_rank(capped=True)
        ids = ids or (rk is None and not flat_only)
        isect_ids = torch.empty(capacity, dtype=torch.int64, device=dev) if ids else None
        flatten_ids = torch.empty(capacity, dtype=torch.int32, device=dev) \
            if (ids or flat_only) else None
        counts = torch.empty(4, dtype=torch.int64, device=dev)  # written by the emission
        # the tile offsets too (as isect_offset_encode with _n_isects_device=counts)
        self.offsets = torch.empty((C, tile_height, tile_width), dtype=torch.int32, device=dev)
        if status is not None:
            assert status.dtype == torch.int32 and status.is_cuda
        ring, slot = (None, None) if report is None else report
        if slot is not None:
            assert slot.dtype == torch.int64 and slot.is_cuda and ring
        if surfel_cull is not None and flat_only and not packed:
            rt, op = (_f32c(t) for t in surfel_cull)
            assert rt.shape == (C, N, 3, 3) and op.shape == (C, N), (rt.shape, op.shape)
            _lib.call("gsplat_hip_isect_write_sorted_capped_surfel", G, N, _ptr(means2d),
                      _ptr(radii), _ptr(depths), _ptr(camera_ids), _ptr(self.tpg), tile_size,
                      tile_width, tile_height, n_bit_tile, n_bit_cam, _ptr(self.ws),
                      _ptr(self.totals), capacity, _ptr(counts), _ptr(status), ring, _ptr(slot),
                      _ptr(ws), ws.numel(), _ptr(flatten_ids), C, _ptr(self.offsets), _ptr(rt),
                      _ptr(op), _stream())
            self.ranks = None
            return self.tpg.view(C, N), None, flatten_ids, counts
        _lib.call("gsplat_hip_isect_write_sorted_capped", G, N, _ptr(means2d), _ptr(radii),
                  _ptr(depths), _ptr(camera_ids), _ptr(self.tpg), tile_size, tile_width,
                  tile_height, n_bit_tile, n_bit_cam, _ptr(self.ws), _ptr(self.totals), capacity,
                  _ptr(counts), _ptr(status), ring, _ptr(slot), _ptr(ws), ws.numel(),
                  _ptr(isect_ids), _ptr(flatten_ids), C, _ptr(self.offsets),
                  *(_ptr(t) for t in (rk or (None, None))), _stream())
        self.ranks = rk
        tpg = self.tpg if packed else self.tpg.view(C, N)
        return tpg, isect_ids, flatten_ids, counts


@torch.no_grad()
def isect_offset_encode(isect_ids: Tensor, C: int, tile_width: int, tile_height: int,
                        _n_isects_device: Optional[Tensor] = None) -> Tensor:
    """First sorted isect index of every tile, i32 [C, tile_height, tile_width]
    (isect_offset.py:8-33).  `_n_isects_device` (private): the count on the
    device when isect_ids is a capacity-sized array (finish_capped)."""
    _dev_check(isect_ids)
    isect_ids = isect_ids.contiguous()
    offsets = torch.empty((C, tile_height, tile_width), dtype=torch.int32, device=isect_ids.device)
    _lib.call("gsplat_hip_isect_offsets", isect_ids.numel(), _ptr(_n_isects_device),
              _ptr(isect_ids), C, tile_width, tile_height, _ptr(offsets), _stream())
    return offsets


# ====================================================== spherical harmonics ==
def _coeff_rows(coeffs: Tensor) -> Tuple[Tensor, int]:
    """[..., K, 3] coefficients -> (contiguous storage, n_coeff_rows).  A
    [N,K,3] tensor expanded to [C,N,K,3] (rendering.py:404) is read in place."""
    if coeffs.dim() == 4 and coeffs.size(0) > 1 and coeffs.stride(0) == 0 \
            and coeffs[0].is_contiguous() and coeffs.dtype == torch.float32:
        return coeffs[0], coeffs.size(1)
    c = _f32c(coeffs)
    return c, c.numel() // (c.shape[-2] * c.shape[-1])


class _SphericalHarmonics(torch.autograd.Function):
    """Spherical harmonics (gsplat/triton_impl/_wrapper.py:552-593)."""

    @staticmethod
    def forward(ctx, sh_degree, dirs, coeffs, masks, block_size=None, coeffs_rest=None):
        dirs = _f32c(dirs)
        base, n_rows = _coeff_rows(coeffs)
        rest = None
        if coeffs_rest is not None:  # split (sh0 [..,1,3], shN [..,K-1,3]) form
            rest, n_rows_r = _coeff_rows(coeffs_rest)
            assert n_rows_r == n_rows and coeffs.shape[-2] == 1, (coeffs.shape, coeffs_rest.shape)
        _dev_check(dirs, base, rest)
        K = coeffs.shape[-2] + (0 if rest is None else coeffs_rest.shape[-2])
        n = dirs.numel() // 3
        m = None if masks is None else masks.to(torch.bool).contiguous()
        colors = torch.empty(*dirs.shape[:-1], 3, device=dirs.device, dtype=torch.float32)
        _lib.call("gsplat_hip_sh_fwd", int(sh_degree), n, n_rows, K, _ptr(dirs), _ptr(base),
                  _ptr(rest), _ptr(m), _ptr(colors), _stream())
        ctx.save_for_backward(dirs, base, rest, m)
        ctx.sh_degree, ctx.n_rows, ctx.K = int(sh_degree), n_rows, K
        ctx.coeff_shape = coeffs.shape
        ctx.rest_shape = None if coeffs_rest is None else coeffs_rest.shape
        return colors

    @staticmethod
    def backward(ctx, v_colors):
        dirs, base, rest, m = ctx.saved_tensors
        K = ctx.K
        n = dirs.numel() // 3
        v_colors = _f32c(v_colors)
        lead = dirs.shape[:-1]
        if rest is None:
            v_coeffs = torch.empty(*lead, K, 3, device=dirs.device)
            v_rest = None
        else:
            v_coeffs = torch.empty(*lead, 1, 3, device=dirs.device)
            v_rest = torch.empty(*lead, K - 1, 3, device=dirs.device)
        want_dirs = ctx.needs_input_grad[1]
        v_dirs = torch.empty_like(dirs) if want_dirs else None
        _lib.call("gsplat_hip_sh_bwd", ctx.sh_degree, n, ctx.n_rows, K, _ptr(dirs), _ptr(base),
                  _ptr(rest), _ptr(m), _ptr(v_colors), _ptr(v_coeffs), _ptr(v_rest),
                  _ptr(v_dirs), _stream())
        v_rest = None if v_rest is None else v_rest.view(ctx.rest_shape)
        return None, v_dirs, v_coeffs.view(ctx.coeff_shape), None, None, v_rest


def spherical_harmonics(
    degrees_to_use: int,
    dirs: Tensor,  # [..., 3]
    coeffs: Tensor,  # [..., K, 3]
    masks: Optional[Tensor] = None,
    block_size: int = None,
) -> Tensor:
    """Computes spherical harmonics colours [..., 3] (_wrapper.py:596-620).

    Extension: `coeffs` may also be the pair (sh0 [...,1,3], shN [...,K-1,3])
    as the trainer stores them; it is read in place instead of concatenated."""
    rest = None
    if isinstance(coeffs, (tuple, list)):
        coeffs, rest = coeffs
        assert coeffs.shape[-2] == 1 and rest.shape[:-2] == coeffs.shape[:-2], \
            (coeffs.shape, rest.shape)
    K = coeffs.shape[-2] + (0 if rest is None else rest.shape[-2])
    assert (degrees_to_use + 1) ** 2 <= K, (coeffs.shape, K)
    assert dirs.shape[:-1] == coeffs.shape[:-2], (dirs.shape, coeffs.shape)
    assert dirs.shape[-1] == 3, dirs.shape
    assert coeffs.shape[-1] == 3, coeffs.shape
    if masks is not None:
        assert masks.shape == dirs.shape[:-1], masks.shape
    return _SphericalHarmonics.apply(degrees_to_use, dirs, coeffs, masks, block_size, rest)


class StepFusion:
    """The optimizer work one training step folds into its own backward,
    handed EXPLICITLY to the forward calls that create the autograd nodes
    (`rasterization(_fusion=...)`, `strategy.activate(..., fusion=...)`), so
    nothing is armed in module state: a render or backward that was not given
    this object is never affected.

    sh_adam -- a ShAdamInBackward: the SH-colour backward applies Adam to the
               SH coefficients in place instead of returning their gradients;
    geom    -- the SH-colour backward hands its dL/dmeans (`v_dirs`) and the
               activation backward its incoming dL/dscales, dL/dopacities
               (`v_scales`, `v_opac`, with the activations `scales`, `opac`)
               to the trainer, whose geometry Adam forms the sums / VJPs
               in-register (gsplat_hip_adam_step_ex).
    Each hand-over happens at most once: a second backward through the same
    nodes (retain_graph) returns ordinary gradients, which the trainer then
    adds as extra terms."""

    def __init__(self, sh_adam: Optional["ShAdamInBackward"] = None, geom: bool = False,
                 geom_adam: Optional["GeomAdamInBackward"] = None):
        self.sh_adam = sh_adam
        self.geom = bool(geom) or geom_adam is not None
        self.geom_adam = geom_adam
        self.v_dirs = None
        self.v_scales = self.v_opac = self.scales = self.opac = None
        self.act_taken = False
        # geom_adam: set in the forward by the nodes whose gradients the
        # projection backward needs (the SH colours' means gradient, the
        # opacities' gradient through _OpacityTap, the activation's output)
        self.expect_v_dirs = False
        self.opac_act = None
        self.opac_tapped = False
        self.v_opac_in = None

    def geom_adam_ready(self) -> bool:
        """The projection backward may run the geometry Adam: armed, not run
        yet, and every gradient it consumes has arrived (autograd runs the SH
        colours' and the opacity tap's backward before the projection's: they
        were created after it; otherwise the step takes the unfused path)."""
        ga = self.geom_adam
        return (ga is not None and not ga.applied and self.opac_act is not None
                and (self.v_dirs is not None or not self.expect_v_dirs)
                and (self.v_opac_in is not None or not self.opac_tapped))

    def take_means_grad(self, v_means: Optional[Tensor]) -> Optional[Tensor]:
        """The SH backward's means gradient: kept here (returns None) when the
        geometry update takes it, else handed back to autograd."""
        if v_means is not None and self.geom and self.v_dirs is None:
            self.v_dirs = v_means
            return None
        return v_means

    def take_activation_grads(self, v_scales, v_opac, scales, opac) -> bool:
        """The activation backward's incoming gradients (True: taken)."""
        if not self.geom or self.act_taken:
            return False
        self.act_taken = True
        self.v_scales, self.v_opac, self.scales, self.opac = v_scales, v_opac, scales, opac
        return True


class GeomAdamInBackward:
    """Arms the next projection backward (C == 1) to apply torch.optim.Adam to
    the four geometry parameters [means, log-scales, quats, logits] (the
    trainer's order and learning rates) in place, from the gradients the
    trainer's FusedAdam would have formed (gsplat_hip_projection_bwd_adam):
    the optimizer step fused into its producer, as ShAdamInBackward does for
    the SH rows.  `applied` tells the caller whether it ran; the activation
    backward then returns nothing (its gradients were consumed)."""

    def __init__(self, params, exp_avgs, exp_avg_sqs, lrs, betas, eps, step, hyper=None,
                 skip=None):
        assert len(params) == len(exp_avgs) == len(exp_avg_sqs) == len(lrs) == 4
        self.params, self.exp_avgs, self.exp_avg_sqs = list(params), list(exp_avgs), \
            list(exp_avg_sqs)
        self.lrs, self.betas, self.eps, self.step = [float(x) for x in lrs], betas, eps, step
        self.hyper, self.skip = hyper, skip  # captured step: device factors f32[8], void flag
        self.applied = False

    def run(self, means, quats, scales, viewmats, Ks, width, height, eps2d, radii, conics,
            v_means2d, v_depths, v_conics, fusion):
        N = means.shape[0]
        for t in self.params + self.exp_avgs + self.exp_avg_sqs:
            assert t.is_contiguous() and t.dtype == torch.float32
        assert [t.shape[0] for t in self.params] == [N] * 4
        P = ctypes.c_void_p * 4
        v_opac = fusion.v_opac_in
        _lib.call("gsplat_hip_projection_bwd_adam", N, _ptr(means), _ptr(quats), _ptr(scales),
                  _ptr(viewmats), _ptr(Ks), int(width), int(height), float(eps2d), _ptr(radii),
                  _ptr(conics), _ptr(v_means2d), _ptr(v_depths), _ptr(v_conics),
                  _ptr(fusion.v_dirs), _ptr(v_opac), _ptr(fusion.opac_act),
                  P(*[t.data_ptr() for t in self.params]),
                  P(*[t.data_ptr() for t in self.exp_avgs]),
                  P(*[t.data_ptr() for t in self.exp_avg_sqs]),
                  (ctypes.c_float * 4)(*self.lrs), float(self.betas[0]), float(self.betas[1]),
                  float(self.eps), int(self.step), _ptr(self.hyper), _ptr(self.skip), _stream())
        self.applied = True


    def run_2dgs(self, means, quats, scales, viewmats, Ks, radii, ray_transforms, v_means2d,
                 v_depths, v_normals, v_ray_transforms, fusion):
        """The 2DGS projection backward's form (gsplat_hip_projection_2dgs_bwd_adam)."""
        N = means.shape[0]
        for t in self.params + self.exp_avgs + self.exp_avg_sqs:
            assert t.is_contiguous() and t.dtype == torch.float32
        assert [t.shape[0] for t in self.params] == [N] * 4
        P = ctypes.c_void_p * 4
        _lib.call("gsplat_hip_projection_2dgs_bwd_adam", N, _ptr(means), _ptr(quats),
                  _ptr(scales), _ptr(viewmats), _ptr(Ks), _ptr(radii), _ptr(ray_transforms),
                  _ptr(v_means2d), _ptr(v_depths), _ptr(v_normals), _ptr(v_ray_transforms),
                  _ptr(fusion.v_dirs), _ptr(fusion.v_opac_in), _ptr(fusion.opac_act),
                  P(*[t.data_ptr() for t in self.params]),
                  P(*[t.data_ptr() for t in self.exp_avgs]),
                  P(*[t.data_ptr() for t in self.exp_avg_sqs]),
                  (ctypes.c_float * 4)(*self.lrs), float(self.betas[0]), float(self.betas[1]),
                  float(self.eps), int(self.step), _ptr(self.hyper), _ptr(self.skip), _stream())
        self.applied = True


class _OpacityTap(torch.autograd.Function):
    """opacities[None] for one camera, whose backward also hands the incoming
    dL/dopacities to the step's StepFusion (the geometry Adam in the
    projection backward reads it; autograd runs this node's backward first:
    it is created after the projection)."""

    @staticmethod
    def forward(ctx, opacities, fusion):
        ctx.fusion = fusion
        fusion.opac_tapped = True
        return opacities.view(1, -1)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            g = _f32c(g)
            ctx.fusion.v_opac_in = g
            return g.view(-1), None
        return None, None


class ShAdamInBackward:
    """Arms the next SH-colour backward (C == 1, coefficients [N,1,3] +
    [N,15,3]) to apply torch.optim.Adam to these coefficient tensors in place
    instead of returning their gradients (gsplat_hip_sh_colors_bwd_adam): the
    trainer's optimizer step for the SH groups fused into their producer.
    `applied` tells the caller whether it ran (else: take the normal step)."""

    def __init__(self, coeffs, coeffs_rest, m0, v0, m_rest, v_rest, lr0, lr_rest, betas, eps,
                 step, hyper=None, skip=None):
        self.coeffs, self.coeffs_rest = coeffs, coeffs_rest
        self.moments = (m0, v0, m_rest, v_rest)
        self.lr0, self.lr_rest, self.betas, self.eps, self.step = lr0, lr_rest, betas, eps, step
        # captured-step form: the step's factors {lr0 / bc1, lr_rest / bc1,
        # 1 / sqrt(bc2)} in a device f32[3] view, and a device i32 void-step
        # flag (gsplat_hip_sh_colors_bwd_adam_dev)
        self.hyper, self.skip = hyper, skip
        self.applied = False

    def matches(self, base, rest, C, N, K, n_rows, degree):
        # degree 3 only: the staged kernel of the unfused backward at K == 16,
        # so the two paths are bit-identical (lower degrees of the SH schedule
        # take the unfused path); C cameras sharing the coefficient rows (a
        # Gaussian-sharded render) sum their gradients in the kernel first
        return (not self.applied and rest is not None and K == 16 and n_rows == N
                and degree == 3 and base.data_ptr() == self.coeffs.data_ptr()
                and rest.data_ptr() == self.coeffs_rest.data_ptr()
                and self.coeffs.is_contiguous() and self.coeffs_rest.is_contiguous())


class _SHColors(torch.autograd.Function):
    """rasterization()'s SH colour path in one kernel each way
    (gsplat/rendering.py:396-406): clamp_min(SH(means - campos) + 0.5, 0)
    with radii masking.  Differentiable w.r.t. means and the coefficients
    (viewmats must not require grad -- the caller falls back otherwise).
    `fusion`: the training step's StepFusion or None."""

    @staticmethod
    def forward(ctx, sh_degree, means, viewmats, coeffs, coeffs_rest, radii, fusion=None):
        ctx.fusion = fusion
        if fusion is not None and fusion.geom and ctx.needs_input_grad[1]:
            fusion.expect_v_dirs = True  # this backward hands dL/dmeans to the fusion
        means, viewmats = _f32c(means), _f32c(viewmats)
        base, n_rows = _coeff_rows(coeffs)
        rest = None
        if coeffs_rest is not None:
            rest, n_rows_r = _coeff_rows(coeffs_rest)
            assert n_rows_r == n_rows and coeffs.shape[-2] == 1, (coeffs.shape, coeffs_rest.shape)
        radii = radii.to(torch.int32).contiguous()
        _dev_check(means, viewmats, base, rest, radii)
        C, N = radii.shape
        K = coeffs.shape[-2] + (0 if rest is None else coeffs_rest.shape[-2])
        colors = torch.empty(C, N, 3, device=means.device, dtype=torch.float32)
        _lib.call("gsplat_hip_sh_colors_fwd", int(sh_degree), C, N, n_rows, K, _ptr(means),
                  _ptr(viewmats), _ptr(base), _ptr(rest), _ptr(radii), _ptr(colors), _stream())
        ctx.save_for_backward(means, viewmats, base, rest, radii)
        ctx.sh_degree, ctx.n_rows, ctx.K = int(sh_degree), n_rows, K
        ctx.coeff_shape = coeffs.shape
        ctx.rest_shape = None if coeffs_rest is None else coeffs_rest.shape
        return colors

    @staticmethod
    def backward(ctx, v_colors):
        means, viewmats, base, rest, radii = ctx.saved_tensors
        C, N = radii.shape
        K = ctx.K
        v_colors = _f32c(v_colors)
        dev = means.device
        want_means = ctx.needs_input_grad[1]
        # C == 1: a plain [N, 3] tensor (same bytes as [1, N, 3]), so autograd's
        # gradient accumulation can take it over instead of copying a view
        fusion = ctx.fusion
        fa = None if fusion is None else fusion.sh_adam
        fused_adam = fa is not None and fa.matches(base, rest, C, N, K, ctx.n_rows, ctx.sh_degree)
        # C cameras sharing the coefficient rows (the trainer's layout): the
        # sums over the cameras formed in the kernel (gsplat_hip_sh_colors_bwd_sum)
        shared = (C > 1 and rest is not None and K == 16 and ctx.n_rows == N
                  and ctx.sh_degree <= 3 and len(ctx.coeff_shape) == 3)
        v_dirs = (torch.empty(N, 3, device=dev) if C == 1 or fused_adam or shared else
                  torch.empty(C, N, 3, device=dev)) if want_means else None
        if fused_adam:
            m0, v0, mr, vr = fa.moments
            if fa.hyper is not None:
                _lib.call("gsplat_hip_sh_colors_bwd_adam_dev", ctx.sh_degree, C, N, _ptr(means),
                          _ptr(viewmats), _ptr(base), _ptr(rest), _ptr(radii), _ptr(v_colors),
                          _ptr(v_dirs), _ptr(m0), _ptr(v0), _ptr(mr), _ptr(vr), _ptr(fa.hyper),
                          ctypes.c_float(fa.betas[0]), ctypes.c_float(fa.betas[1]),
                          ctypes.c_float(fa.eps), _ptr(fa.skip), _stream())
            else:
                _lib.call("gsplat_hip_sh_colors_bwd_adam", ctx.sh_degree, C, N, _ptr(means),
                          _ptr(viewmats), _ptr(base), _ptr(rest), _ptr(radii), _ptr(v_colors),
                          _ptr(v_dirs), _ptr(m0), _ptr(v0), _ptr(mr), _ptr(vr),
                          ctypes.c_float(fa.lr0), ctypes.c_float(fa.lr_rest),
                          ctypes.c_float(fa.betas[0]), ctypes.c_float(fa.betas[1]),
                          ctypes.c_float(fa.eps), int(fa.step), _stream())
            fa.applied = True
            return (None, fusion.take_means_grad(v_dirs), None, None, None, None, None)
        if shared:
            v_base = torch.empty(N, 1, 3, device=dev)
            v_rest_s = torch.empty(N, K - 1, 3, device=dev)
            _lib.call("gsplat_hip_sh_colors_bwd_sum", ctx.sh_degree, C, N, _ptr(means),
                      _ptr(viewmats), _ptr(base), _ptr(rest), _ptr(radii), _ptr(v_colors),
                      _ptr(v_base), _ptr(v_rest_s), _ptr(v_dirs), _stream())
            v_means = v_dirs
            if v_means is not None and fusion is not None:
                v_means = fusion.take_means_grad(v_means)
            return (None, v_means, None, v_base.view(ctx.coeff_shape),
                    v_rest_s.view(ctx.rest_shape), None, None)
        if rest is None:
            v_coeffs = torch.empty(C, N, K, 3, device=dev)
            v_rest = None
        else:
            v_coeffs = torch.empty(C, N, 1, 3, device=dev)
            v_rest = torch.empty(C, N, K - 1, 3, device=dev)
        _lib.call("gsplat_hip_sh_colors_bwd", ctx.sh_degree, C, N, ctx.n_rows, K, _ptr(means),
                  _ptr(viewmats), _ptr(base), _ptr(rest), _ptr(radii), _ptr(v_colors),
                  _ptr(v_coeffs), _ptr(v_rest), _ptr(v_dirs), _stream())
        v_means = None
        if want_means:
            v_means = v_dirs if C == 1 else v_dirs.sum(0)
            if fusion is not None:
                v_means = fusion.take_means_grad(v_means)
        def fold(v, shape):  # [C,N,..] -> the input's shape (sum over cameras)
            if v is None:
                return None
            if len(shape) == 3:  # shared [N,K,3] coefficients
                v = v[0] if C == 1 else v.sum(0)
            return v.view(shape)
        return (None, v_means, None, fold(v_coeffs, ctx.coeff_shape), fold(v_rest, ctx.rest_shape),
                None, None)


def sh_colors(sh_degree: int, means: Tensor, viewmats: Tensor, coeffs, radii: Tensor,
              fusion: Optional[StepFusion] = None) -> Tensor:
    """colors [C,N,3] = clamp_min(SH(means - campos) + 0.5, 0), radii-masked:
    the colour computation of rendering.rasterization (rendering.py:396-406)
    fused.  `coeffs`: [N,K,3] / [C,N,K,3] or the pair (sh0, shN).  `fusion`:
    the training step's StepFusion (optimizer work folded into the backward)."""
    rest = None
    if isinstance(coeffs, (tuple, list)):
        coeffs, rest = coeffs
    return _SHColors.apply(sh_degree, means, viewmats, coeffs, rest, radii, fusion)


# ============================================================ rasterization ==
class _RasterizeToPixels(torch.autograd.Function):
    """Rasterize Gaussians (gsplat/triton_impl/_wrapper.py:42-182)."""

    @staticmethod
    def forward(ctx, means2d, conics, colors, opacities, backgrounds, masks, width, height,
                tile_size, isect_offsets, flatten_ids, absgrad, block_size=8, visible=None,
                records=None, n_dev=None, ranks=None):
        ctx.means2d_in = means2d if absgrad else None  # receives .absgrad (_wrapper.py:156)
        ctx.set_materialize_grads(False)  # alphas without a loss: None, not zeros
        means2d, conics, colors, opacities, backgrounds = (
            _f32c(x) for x in (means2d, conics, colors, opacities, backgrounds))
        _dev_check(means2d, conics, colors, opacities, isect_offsets, flatten_ids)
        isect_offsets = isect_offsets.to(torch.int32).contiguous()
        flatten_ids = flatten_ids.to(torch.int32).contiguous()
        m = None if masks is None else masks.to(torch.bool).contiguous()
        C, th, tw = isect_offsets.shape
        D = colors.shape[-1]
        dev = means2d.device
        render_colors = torch.empty((C, height, width, D), device=dev)
        render_alphas = torch.empty((C, height, width, 1), device=dev)
        last_ids = torch.empty((C, height, width), dtype=torch.int32, device=dev)
        # compositing state at the chunk boundaries of long tiles, for the
        # chunked backward (csrc/rasterize16.hip); empty when not used
        sb = int(_lib.query("gsplat_hip_rasterize_fwd_state_bytes", C, D, tile_size, tw, th,
                            flatten_ids.numel()))
        state = torch.empty(sb // 4, dtype=torch.float32, device=dev)
        # one 64-B render record per Gaussian for the 16x16 kernels' gathers
        # (rasterization() may have packed them already, before its isect sync)
        if records is None:
            records = pack_render_records(means2d, conics, colors, opacities, tile_size, visible,
                                          ranks)
        rf = 1 if records.numel() else 0
        # rank-indexed records (ranks = (rank_ids, vis_rank), packed by rank):
        # the kernels walk the isects' ranks instead of their Gaussians
        vis_rank = None
        kernel_ids = flatten_ids
        if ranks is not None and rf and visible is not None:
            kernel_ids, vis_rank = ranks
        if sb:  # dispatch order into the state, outside the timed rasterizer launch
            _lib.call("gsplat_hip_rasterize_prepare", C, D, tile_size, tw, th, _ptr(isect_offsets),
                      flatten_ids.numel(), _ptr(n_dev), _ptr(state), sb, _stream())
        with _Timed("rasterize_fwd"):
            _lib.call("gsplat_hip_rasterize_fwd", C, D, width, height, tile_size, tw, th,
                      _ptr(means2d), _ptr(conics), _ptr(colors), _ptr(opacities),
                      _ptr(backgrounds), _ptr(m), _ptr(isect_offsets), flatten_ids.numel(),
                      _ptr(n_dev), _ptr(kernel_ids), _ptr(render_colors), _ptr(render_alphas),
                      _ptr(last_ids), _ptr(records) if rf else 0, _ptr(state) if sb else 0, sb,
                      _stream())
        ctx.save_for_backward(means2d, conics, colors, opacities, backgrounds, m, isect_offsets,
                              kernel_ids, render_alphas, last_ids, render_colors, state, records,
                              vis_rank)
        ctx.width, ctx.height, ctx.tile_size, ctx.absgrad = width, height, tile_size, absgrad
        ctx.n_dev = n_dev
        # tiles_per_gauss: the backward zeroes / reads only those rows
        ctx.visible = None if visible is None else visible.to(torch.int32).contiguous()
        if ctx.visible is not None and ctx.visible.numel() != opacities.numel():
            ctx.visible = None
        return render_colors, render_alphas

    @staticmethod
    def backward(ctx, v_render_colors, v_render_alphas):
        (means2d, conics, colors, opacities, backgrounds, m, isect_offsets, flatten_ids,
         render_alphas, last_ids, render_colors, state, records, vis_rank) = ctx.saved_tensors
        C, th, tw = isect_offsets.shape
        D = colors.shape[-1]
        G = opacities.numel()
        if v_render_colors is None:
            v_render_colors = torch.zeros_like(render_colors)
        v_render_colors = _f32c(v_render_colors)
        v_render_alphas = _f32c(v_render_alphas)  # None: alphas unused (null in the ABI)
        v_means2d = torch.empty_like(means2d)
        v_conics = torch.empty_like(conics)
        v_colors = torch.empty_like(colors)
        v_opacities = torch.empty_like(opacities)
        v_abs = torch.empty_like(means2d) if ctx.absgrad else None
        wsb = int(_lib.query("gsplat_hip_rasterize_bwd_workspace_bytes", G, D, ctx.tile_size,
                             int(bool(ctx.absgrad)), C, tw, th, flatten_ids.numel()))
        ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=means2d.device)
        with _Timed("rasterize_bwd"):
            _lib.call("gsplat_hip_rasterize_bwd", C, G, D, ctx.width, ctx.height, ctx.tile_size,
                      tw, th, _ptr(means2d), _ptr(conics), _ptr(colors), _ptr(opacities),
                      _ptr(backgrounds), _ptr(m), _ptr(isect_offsets), flatten_ids.numel(),
                      _ptr(ctx.n_dev), _ptr(flatten_ids), _ptr(render_alphas), _ptr(last_ids),
                      _ptr(v_render_colors), _ptr(v_render_alphas), _ptr(v_means2d),
                      _ptr(v_conics), _ptr(v_colors), _ptr(v_opacities), _ptr(v_abs),
                      _ptr(render_colors), _ptr(records) if records.numel() else 0,
                      _ptr(state) if state.numel() else 0, state.numel() * 4, _ptr(ws), wsb,
                      _ptr(ctx.visible), _ptr(vis_rank if ctx.visible is not None else None),
                      _stream())
        if ctx.absgrad:
            ctx.means2d_in.absgrad = v_abs
        v_backgrounds = None
        if ctx.needs_input_grad[4]:
            v_backgrounds = (v_render_colors * (1.0 - render_alphas)).sum(dim=(1, 2))
        return (v_means2d, v_conics, v_colors, v_opacities, v_backgrounds,
                None, None, None, None, None, None, None, None, None, None, None, None)


def rasterize_to_pixels(
    means2d: Tensor,  # [C, N, 2] or [nnz, 2]
    conics: Tensor,  # [C, N, 3] or [nnz, 3]
    colors: Tensor,  # [C, N, channels] or [nnz, channels]
    opacities: Tensor,  # [C, N] or [nnz]
    image_width: int,
    image_height: int,
    tile_size: int,
    isect_offsets: Tensor,  # [C, tile_height, tile_width]
    flatten_ids: Tensor,  # [n_isects]
    backgrounds: Optional[Tensor] = None,  # [C, channels]
    masks: Optional[Tensor] = None,  # [C, tile_height, tile_width]
    packed: bool = False,
    absgrad: bool = False,
    block_size: int = 8,
) -> Tuple[Tensor, Tensor]:
    """Rasterizes Gaussians to pixels (_wrapper.py:185-297).

    Returns render_colors [C,H,W,channels] and render_alphas [C,H,W,1].
    Channel counts outside {1,2,3,4,8,16,32} are zero-padded to the next one;
    above 32 they are rendered in chunks of 32."""
    return _rasterize_to_pixels(means2d, conics, colors, opacities, image_width, image_height,
                                tile_size, isect_offsets, flatten_ids, backgrounds, masks, packed,
                                absgrad, block_size)


@contextlib.contextmanager
def fwd_split(div: Optional[int], threshold: Optional[int] = None):
    """The split forward's threshold divisor (gsplat_hip_set_fwd_split_div)
    and fixed threshold (gsplat_hip_set_fwd_split_threshold: > 0 always the
    split-capable variant with that threshold, 0 never split) for the renders
    queued inside the block only; the previous values are restored after it,
    so a trainer's choice does not leak into other rasterization() calls of
    the process.  None: leave that one alone (div 0 as well)."""
    old_div = int(_lib.query("gsplat_hip_set_fwd_split_div", int(div))) if div else None
    old_thr = (int(_lib.query("gsplat_hip_set_fwd_split_threshold", int(threshold)))
               if threshold is not None else None)
    try:
        yield
    finally:
        if old_thr is not None:
            _lib.query("gsplat_hip_set_fwd_split_threshold", old_thr)
        if old_div is not None:
            _lib.query("gsplat_hip_set_fwd_split_div", old_div)


def max_tile_isects(meta: dict) -> int:
    """The largest tile's isect count of a render (its meta's offsets and ids)."""
    offs = meta["isect_offsets"].flatten().long()
    n = int(meta["isect_counts"][0]) if "isect_counts" in meta else meta["flatten_ids"].numel()
    if n <= 0 or offs.numel() == 0:
        return 0
    ends = torch.cat([offs[1:], torch.tensor([n], device=offs.device)])
    return int((ends - offs).max())


def fwd_split_threshold(n_isects: int) -> int:
    """gsplat_hip_fwd_split_threshold: isects above which a tile splits with
    the divisor in effect (-1: splitting off)."""
    return int(_lib.query("gsplat_hip_fwd_split_threshold", int(n_isects)))


@torch.no_grad()
def forward_termination_ratio(colors: Tensor, meta: dict, width: int, height: int) -> float:
    """n_eff / n_isects of a 3DGS render (colors from rasterization() with a
    gradient to compute): n_eff = sum over tiles of min(range end, the tile's
    largest last id + 1) - range start, from the forward's own last ids (the
    autograd node's saved tensors).  1.0 when the node is not found."""
    offs = meta["isect_offsets"].flatten().long()
    n = int(meta["isect_counts"][0]) if "isect_counts" in meta else meta["flatten_ids"].numel()
    if n <= 0:
        return 1.0
    node = colors.grad_fn
    while node is not None and type(node).__name__ != "_RasterizeToPixelsBackward":
        node = node.next_functions[0][0] if node.next_functions else None
    if node is None:
        return 1.0
    last = node.saved_tensors[9]  # (..., render_alphas, last_ids, ...): see _RasterizeToPixels
    ts, tw, th = meta["tile_size"], meta["tile_width"], meta["tile_height"]
    lp = torch.nn.functional.pad(last[0], (0, tw * ts - width, 0, th * ts - height))
    tmax = lp.view(th, ts, tw, ts).amax(dim=(1, 3)).flatten().long()
    ends = torch.cat([offs[1:], torch.tensor([n], device=offs.device)])
    n_eff = int(torch.clamp(torch.minimum(ends, tmax + 1) - offs, min=0).sum())
    return n_eff / n


def pack_render_records(means2d, conics, colors, opacities, tile_size, visible=None,
                        ranks=None) -> Tensor:
    """The 16x16 rasterizer's render records (gsplat_hip_rasterize_pack_records):
    one 64-B row [x, y, conic, opacity, colour] per Gaussian, only the rows
    whose `visible` count (tiles_per_gauss) is > 0 written.  Empty when the
    configuration has no record path (then the kernels gather the arrays).
    `ranks` = (rank_ids, vis_rank) of the sorted emission (with `visible`):
    the row of Gaussian g is vis_rank[g]."""
    D = colors.shape[-1]
    rf = int(_lib.query("gsplat_hip_rasterize_record_floats", D, tile_size)) if RECORDS else 0
    G = opacities.numel()
    if G * rf * 4 >= 2 ** 31:  # buffer-load offsets are 32-bit: gather the arrays instead
        rf = 0
    records = torch.empty(G * rf if rf else 0, dtype=torch.float32, device=means2d.device)
    if rf:
        means2d, conics, colors, opacities = (_f32c(x) for x in (means2d, conics, colors,
                                                                 opacities))
        vis = None if visible is None else visible.to(torch.int32).contiguous()
        assert vis is None or vis.numel() == G, (vis.shape, G)
        vr = ranks[1] if (ranks is not None and vis is not None) else None
        _lib.call("gsplat_hip_rasterize_pack_records", G, D, _ptr(means2d), _ptr(conics),
                  _ptr(colors), _ptr(opacities), _ptr(vis), _ptr(vr), _ptr(records), _stream())
    return records


def _rasterize_to_pixels(means2d, conics, colors, opacities, image_width, image_height, tile_size,
                         isect_offsets, flatten_ids, backgrounds=None, masks=None, packed=False,
                         absgrad=False, block_size=8, visible=None, records=None,
                         n_isects_device=None, ranks=None):
    """rasterize_to_pixels with rasterization()'s private hints: `visible`
    ([C,N] tiles_per_gauss: only those Gaussians' render records are packed)
    and `records` (already packed by pack_render_records for these exact
    colours; used when no channel padding or chunking applies), and
    `n_isects_device` (flatten_ids is a capacity-sized array, finish_capped)."""
    if n_isects_device is not None:
        assert tile_size == 16, "a device isect count needs 16x16 tiles"
    C = isect_offsets.size(0)
    device = means2d.device
    if packed:
        nnz = means2d.size(0)
        assert means2d.shape == (nnz, 2), means2d.shape
        assert conics.shape == (nnz, 3), conics.shape
        assert colors.shape[0] == nnz, colors.shape
        assert opacities.shape == (nnz,), opacities.shape
    else:
        N = means2d.size(1)
        assert means2d.shape == (C, N, 2), means2d.shape
        assert conics.shape == (C, N, 3), conics.shape
        assert colors.shape[:2] == (C, N), colors.shape
        assert opacities.shape == (C, N), opacities.shape
    if backgrounds is not None:
        assert backgrounds.shape == (C, colors.shape[-1]), backgrounds.shape
    if masks is not None:
        assert masks.shape == isect_offsets.shape, masks.shape

    channels = colors.shape[-1]
    if channels > 512 or channels == 0:
        raise ValueError(f"Unsupported number of color channels: {channels}")
    tile_height, tile_width = isect_offsets.shape[1:3]
    assert tile_height * tile_size >= image_height, \
        f"Assert Failed: {tile_height} * {tile_size} >= {image_height}"
    assert tile_width * tile_size >= image_width, \
        f"Assert Failed: {tile_width} * {tile_size} >= {image_width}"

    def run(cols, bgs):
        D = cols.shape[-1]
        Dp = next(d for d in _SUPPORTED_D if d >= D)
        if Dp != D:
            cols = torch.cat([cols, torch.zeros(*cols.shape[:-1], Dp - D, device=device)], -1)
            if bgs is not None:
                bgs = torch.cat([bgs, torch.zeros(*bgs.shape[:-1], Dp - D, device=device)], -1)
        rc, ra = _RasterizeToPixels.apply(means2d, conics, cols, opacities, bgs, masks,
                                          image_width, image_height, tile_size, isect_offsets,
                                          flatten_ids, absgrad, block_size, visible,
                                          records if Dp == D and cols is colors else None,
                                          n_isects_device, ranks)
        return (rc[..., :D] if Dp != D else rc), ra

    if channels <= 32:
        render_colors, render_alphas = run(colors, backgrounds)
    else:
        outs = []
        render_alphas = None
        for i in range(0, channels, 32):
            rc, ra = run(colors[..., i:i + 32],
                         None if backgrounds is None else backgrounds[..., i:i + 32])
            outs.append(rc)
            render_alphas = ra if render_alphas is None else render_alphas
        render_colors = torch.cat(outs, dim=-1)
    return render_colors, render_alphas
