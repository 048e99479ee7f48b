"""Record the reference's public signatures of the drop-in surface as data
(tests/golden/signatures.json) for tests/test_signatures.py.

Run in the build container only (needs /root/reference):

    python tests/golden/make_signatures.py

Imports the reference modules under make_golden.py's shims
and stores, per function, its parameters as [name, kind, default repr].
Nothing of the reference's text is stored: names and defaults only.
"""

import importlib
import inspect
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402,F401  (installs the shims, puts /root/reference on sys.path)

FUNCS = {
    # the five Triton-backend functions rendering.py imports (SURVEY §8 b)
    "gsplat.triton_impl._wrapper": ["fully_fused_projection", "rasterize_to_pixels",
                                    "spherical_harmonics"],
    "gsplat.triton_impl.isect_tiles": ["isect_tiles"],
    "gsplat.triton_impl.isect_offset": ["get_isect_offsets"],  # = isect_offset_encode
    # 2DGS and the CUDA-only extras the build also replaces (§8 f2-f4)
    "gsplat.cuda._wrapper": ["fully_fused_projection_2dgs", "rasterize_to_pixels_2dgs",
                             "quat_scale_to_covar_preci", "rasterize_to_indices_in_range",
                             "rasterize_to_indices_in_range_2dgs"],
    "gsplat.rendering": ["rasterization", "rasterization_2dgs"],
    "gsplat.distributed": ["all_gather_int32", "all_to_all_int32", "all_gather_tensor_list",
                           "all_to_all_tensor_list"],
}


def describe(fn):
    out = []
    for p in inspect.signature(fn).parameters.values():
        d = None if p.default is inspect.Parameter.empty else repr(p.default)
        out.append([p.name, p.kind.name, d])
    return out


def main():
    sigs = {}
    for mod, names in FUNCS.items():
        m = importlib.import_module(mod)
        for n in names:
            sigs[n] = {"module": mod, "params": describe(getattr(m, n))}
    path = os.path.join(HERE, "signatures.json")
    with open(path, "w") as f:
        json.dump(sigs, f, indent=1, sort_keys=True)
    print(f"wrote {path}: {len(sigs)} functions")


if __name__ == "__main__":
    main()
