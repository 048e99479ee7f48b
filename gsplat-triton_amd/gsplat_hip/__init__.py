"""gsplat_hip -- MI355X (gfx950) backend for the gsplat rasterization hot path.

Exports the backend surface that gsplat/rendering.py imports from
`gsplat.triton_impl._wrapper` (rendering.py:20-27), implemented with
hand-written HIP kernels behind the C ABI in include/gsplat_hip.h, plus a
`rasterization()` front-end mirroring gsplat/rendering.py:44-598.
"""

from ._wrapper import (
    fully_fused_projection,
    isect_offset_encode,
    isect_tiles,
    rasterize_to_pixels,
    spherical_harmonics,
)
from ._wrapper_aux import SelectiveAdam, adam, compute_relocation, quat_scale_to_covar_preci
from ._wrapper_2dgs import fully_fused_projection_2dgs, rasterize_to_pixels_2dgs
from ._wrapper_indices import (
    accumulate,
    accumulate_2dgs,
    rasterize_to_indices_in_range,
    rasterize_to_indices_in_range_2dgs,
)
from .rendering import depth_to_normal, rasterization, rasterization_2dgs

__all__ = [
    "fully_fused_projection",
    "isect_tiles",
    "isect_offset_encode",
    "spherical_harmonics",
    "rasterize_to_pixels",
    "rasterization",
    "fully_fused_projection_2dgs",
    "rasterize_to_pixels_2dgs",
    "rasterization_2dgs",
    "depth_to_normal",
    "quat_scale_to_covar_preci",
    "compute_relocation",
    "adam",
    "SelectiveAdam",
    "rasterize_to_indices_in_range",
    "rasterize_to_indices_in_range_2dgs",
    "accumulate",
    "accumulate_2dgs",
]
__version__ = "0.1.0"
