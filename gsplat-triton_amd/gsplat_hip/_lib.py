"""ctypes binding of libgsplat_hip.so (the C ABI declared in include/gsplat_hip.h).

This is the reference-side binding a maintainer would add next to
gsplat/triton_impl: it replaces the Triton JIT launches and the nvcc-JIT
`radix_sort` extension (gsplat/triton_impl/radix_sort/__init__.py:10-13).
The library is prebuilt in-tree (`make -C gsplat-triton_amd/csrc`); if it is
missing or cannot be loaded every op raises -- there is no fallback path.
"""

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSPLAT_HIP_LIB", os.path.join(_HERE, "libgsplat_hip.so"))
ABI_VERSION = 35

_p = ctypes.c_void_p
_i32 = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float

# name -> (restype, argtypes)
_SIGS = {
    "gsplat_hip_last_error": (ctypes.c_char_p, []),
    "gsplat_hip_abi_version": (_i32, []),
    "gsplat_hip_projection_fwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f, _f, _f,
                                         _f, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_projection_bwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f, _p, _p,
                                         _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_sh_fwd": (_i32, [_i32, _i64, _i64, _i32, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_sh_bwd": (_i32, [_i32, _i64, _i64, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_sh_colors_fwd": (_i32, [_i32, _i32, _i64, _i64, _i32, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_sh_colors_bwd": (_i32, [_i32, _i32, _i64, _i64, _i32, _p, _p, _p, _p, _p, _p, _p,
                                        _p, _p, _p]),
    "gsplat_hip_isect_workspace_bytes": (_i64, [_i64]),
    "gsplat_hip_isect_count": (_i32, [_i64, _p, _p, _i32, _i32, _i32, _p, _p, _p, _p]),
    "gsplat_hip_isect_write": (_i32, [_i64, _i32, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _p,
                                      _p, _p, _p]),
    "gsplat_hip_isect_sorted_workspace_bytes": (_i64, [_i64, _i64, _i32]),
    "gsplat_hip_isect_write_sorted": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _i32, _i32, _i32,
                                             _i32, _i32, _p, _i64, _i64, _p, _i64, _p, _p, _i32,
                                             _p, _p, _p, _p]),
    "gsplat_hip_isect_ranked": (_i32, [_i32, _i32, _i32]),
    "gsplat_hip_isect_tilefirst_workspace_bytes": (_i64, [_i64, _i32, _i32]),
    "gsplat_hip_isect_sorted_capped_workspace_bytes": (_i64, [_i64, _i64, _i32]),
    "gsplat_hip_isect_write_sorted_capped": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _i32, _i32,
                                                    _i32, _i32, _i32, _p, _p, _i64, _p, _p, _p,
                                                    _p, _p, _i64, _p, _p, _i32, _p, _p, _p, _p]),
    "gsplat_hip_isect_write_sorted_capped_surfel": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _i32,
                                                           _i32, _i32, _i32, _i32, _p, _p, _i64,
                                                           _p, _p, _p, _p, _p, _i64, _p, _i32, _p,
                                                           _p, _p, _p]),
    "gsplat_hip_host_mapped_alloc": (_i32, [_i64, _p, _p]),
    "gsplat_hip_host_mapped_free": (_i32, [_p]),
    "gsplat_hip_step_fetch": (_i32, [_p, _i64, _i32, _p, _p, _p]),
    "gsplat_hip_activate_fwd_fetch": (_i32, [_i64, _i64, _p, _p, _p, _p, _p, _i64, _i32, _p, _p,
                                             _p]),
    "gsplat_hip_graph_node_census": (_i32, [_p, _p, _p, _i32]),
    "gsplat_hip_graph_memcpy_census": (_i32, [_p, _p, _i32, _p]),
    "gsplat_hip_status_to_ring": (_i32, [_p, _p, _p, _p]),
    "gsplat_hip_projection_2dgs_bwd_adam": (_i32, [_i32] + [_p] * 18 + [_f] * 3 + [_i32]
                                            + [_p] * 3),
    "gsplat_hip_projection_bwd_adam": (_i32, [_i32, _p, _p, _p, _p, _p, _i32, _i32, _f, _p, _p,
                                              _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _f, _f,
                                              _f, _i32, _p, _p, _p]),
    "gsplat_hip_isect_write_tilefirst": (_i32, [_i64, _i32, _p, _p, _p, _p, _i32, _i32, _i32,
                                                _i32, _i32, _i32, _p, _i64, _p, _i64, _p, _p,
                                                _p]),
    "gsplat_hip_sort_workspace_bytes": (_i64, [_i64]),
    "gsplat_hip_radix_sort": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _i64, _p]),
    "gsplat_hip_isect_offsets": (_i32, [_i64, _p, _p, _i32, _i32, _i32, _p, _p]),
    "gsplat_hip_rasterize_supported_channels": (_i32, [_i32]),
    "gsplat_hip_rasterize_fwd_state_bytes": (_i64, [_i32, _i32, _i32, _i32, _i32, _i64]),
    "gsplat_hip_rasterize_prepare": (_i32, [_i32, _i32, _i32, _i32, _i32, _p, _i64, _p, _p, _i64,
                                            _p]),
    "gsplat_hip_rasterize_record_floats": (_i32, [_i32, _i32]),
    "gsplat_hip_rasterize_pack_records": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_rasterize_fwd": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _p,
                                        _p, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "gsplat_hip_rasterize_bwd_workspace_bytes": (_i64, [_i64, _i32, _i32, _i32, _i32, _i32, _i32,
                                                        _i64]),
    "gsplat_hip_rasterize_bwd": (_i32, [_i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p,
                                        _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p,
                                        _p, _p, _p, _p, _p, _p, _i64, _p, _i64, _p, _p, _p]),
    "gsplat_hip_debug_set_timeline": (_i32, [_p, _i64]),
    "gsplat_hip_debug_set_chunk": (_i32, [_i32]),
    "gsplat_hip_debug_set_flags": (_i32, [_i32]),
    "gsplat_hip_debug_set_fwd_split": (_i32, [_i32]),
    "gsplat_hip_set_fwd_split_div": (_i32, [_i32]),
    "gsplat_hip_set_fwd_split_threshold": (_i32, [_i32]),
    "gsplat_hip_fwd_split_threshold": (_i64, [_i64]),
    "gsplat_hip_ssim_workspace_bytes": (_i64, [_i32, _i32, _i32, _i32]),
    "gsplat_hip_ssim_l1_fwd": (_i32, [_i32, _i32, _i32, _i32, _p, _p, _p, _p, _p]),
    "gsplat_hip_ssim_l1_bwd": (_i32, [_i32, _i32, _i32, _i32, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_l1_ssim_loss_fwd": (_i32, [_i32, _i32, _i32, _i32, _p, _p, _f, _p, _p, _p]),
    "gsplat_hip_l1_ssim_loss_bwd": (_i32, [_i32, _i32, _i32, _i32, _p, _p, _p, _f, _p, _p, _p]),
    "gsplat_hip_l1_ssim_loss_fused_workspace_bytes": (_i64, [_i32, _i32, _i32, _i32]),
    "gsplat_hip_l1_ssim_loss_fused_fwd": (_i32, [_i32, _i32, _i32, _i32, _i32, _p, _p, _p, _f, _p,
                                                  _p, _p, _p]),
    "gsplat_hip_l1_ssim_loss_fused_bwd": (_i32, [_i64, _p, _p, _p, _p]),
    "gsplat_hip_l1_ssim_loss_fused_fwd_ring": (_i32, [_i32, _i32, _i32, _i32, _i32, _p, _p, _p, _f,
                                                       _p, _p, _p, _p, _i64, _p, _p]),
    "gsplat_hip_update_state": (_i32, [_i32, _i64, _p, _p, _f, _f, _p, _p, _p, _p]),
    "gsplat_hip_activate_fwd": (_i32, [_i64, _i64, _p, _p, _p, _p, _p]),
    "gsplat_hip_activate_bwd": (_i32, [_i64, _i64, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_adam_step": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _f, _f, _f, _i32, _p]),
    "gsplat_hip_sh_colors_bwd_adam": (_i32, [_i32, _i32, _i64, _p, _p, _p, _p, _p, _p, _p, _p,
                                             _p, _p, _p, _f, _f, _f, _f, _f, _i32, _p]),
    "gsplat_hip_sh_colors_bwd_adam_dev": (_i32, [_i32, _i32, _i64, _p, _p, _p, _p, _p, _p, _p,
                                                 _p, _p, _p, _p, _p, _f, _f, _f, _p, _p]),
    "gsplat_hip_sh_colors_bwd_sum": (_i32, [_i32, _i32, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                            _p]),
    "gsplat_hip_adam_step_dev": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _p, _p, _f, _f, _f, _p, _p]),
    "gsplat_hip_adam_step_ex": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _p, _p, _f, _f, _f, _i32, _p]),
    "gsplat_hip_densify_workspace_bytes": (_i64, [_i64]),
    "gsplat_hip_densify_plan": (_i32, [_i64, _p, _p, _p, _p, _p, _f, _f, _f, _i32, _f, _f, _f,
                                       _i32, _p, _p, _p]),
    "gsplat_hip_densify_apply": (_i32, [_i64, _p, _p, _p, _i32, _i32, _p, _p, _p, _p, _p, _p, _p,
                                        _p, _p]),
    "gsplat_hip_projection_2dgs_fwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f, _f,
                                              _f, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_projection_2dgs_bwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _p, _p,
                                              _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_projection_2dgs_packed_workspace_bytes": (_i64, [_i32, _i32]),
    "gsplat_hip_projection_2dgs_packed_count": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32,
                                                       _f, _f, _f, _p, _p, _p]),
    "gsplat_hip_projection_2dgs_packed_fwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f,
                                                     _f, _f, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_projection_2dgs_packed_bwd": (_i32, [_i32, _i32, _i64, _p, _p, _p, _p, _p, _i32,
                                                     _i32, _p, _p, _p, _p, _p, _p, _p, _i32, _p,
                                                     _p, _p, _p, _p]),
    "gsplat_hip_rasterize_2dgs_supported_channels": (_i32, [_i32]),
    "gsplat_hip_rasterize_2dgs_fwd": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _p, _p, _p,
                                             _p, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _p, _p,
                                             _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_rasterize_2dgs_record_floats": (_i32, [_i32, _i32]),
    "gsplat_hip_rasterize_2dgs_pack_records": (_i32, [_i64, _i32, _p, _p, _p, _p, _p, _p, _p, _p,
                                                      _p]),
    "gsplat_hip_rasterize_2dgs_bwd_workspace_bytes": (_i64, [_i64, _i32, _i32]),
    "gsplat_hip_rasterize_2dgs_bwd": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32, _i64,
                                             _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64,
                                             _p, _p, _p, _p, _p, _p, _p,
                                             _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                             _p, _p, _i64, _p]),
    "gsplat_hip_quat_scale_to_covar_preci_fwd": (_i32, [_i64, _p, _p, _i32, _p, _p, _p]),
    "gsplat_hip_quat_scale_to_covar_preci_bwd": (_i32, [_i64, _p, _p, _i32, _p, _p, _p, _p, _p]),
    "gsplat_hip_relocation": (_i32, [_i64, _p, _p, _p, _p, _i32, _p, _p, _p]),
    "gsplat_hip_selective_adam": (_i32, [_i64, _i64, _p, _p, _p, _p, _p, _f, _f, _f, _f, _p]),
    "gsplat_hip_mcmc_inject_noise": (_i32, [_i64, _p, _p, _p, _p, _p, ctypes.c_uint64, _i64, _p,
                                            _f, _p, _p, _p]),
    "gsplat_hip_projection_packed_workspace_bytes": (_i64, [_i32, _i32]),
    "gsplat_hip_projection_packed_count": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f,
                                                  _f, _f, _f, _p, _p, _p]),
    "gsplat_hip_projection_packed_fwd": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _i32, _i32, _f, _f,
                                                _f, _f, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "gsplat_hip_projection_packed_bwd": (_i32, [_i32, _i32, _i64, _p, _p, _p, _p, _p, _i32, _i32,
                                                _f, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _p,
                                                _p, _p, _p]),
    "gsplat_hip_rasterize_to_indices_count": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                                     _i32, _i64, _i64, _i64, _p, _p, _p, _p, _p,
                                                     _p, _p, _p]),
    "gsplat_hip_rasterize_to_indices_write": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _i32,
                                                     _i32, _i64, _i64, _i64, _p, _p, _p, _p, _p,
                                                     _p, _p, _p, _p, _p]),
    "gsplat_hip_depth_to_normal": (_i32, [_i32, _i32, _i32, _p, _i64, _p, _p, _i32, _p, _p]),
    "gsplat_hip_rotate3": (_i32, [_i32, _i64, _p, _p, _p, _p]),
    "gsplat_hip_watchdog_arm": (_i32, [ctypes.c_double, ctypes.c_char_p, _i32]),
    "gsplat_hip_watchdog_beat": (_i32, [ctypes.c_char_p]),
    "gsplat_hip_watchdog_set_fallback": (_i32, [_i32, ctypes.c_char_p, _i32]),
    "gsplat_hip_watchdog_disarm": (_i32, []),
}

EXPORTED = tuple(_SIGS)

_lib = None


class GsplatHipError(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes library, raising if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GsplatHipError(
            f"libgsplat_hip.so not found at {LIB_PATH}; build it with "
            "`make -C gsplat-triton_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.gsplat_hip_abi_version()
    if v != ABI_VERSION:
        raise GsplatHipError(f"libgsplat_hip ABI {v} != expected {ABI_VERSION}; rebuild")
    _lib = lib
    return lib


def call(name, *args):
    """Invoke an int-returning entry point and raise on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.gsplat_hip_last_error().decode(errors="replace")
        raise GsplatHipError(f"{name} failed (status {rc}): {msg}")
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)
