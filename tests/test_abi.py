"""CPU-only checks of the C-ABI boundary: the library loads, exports every
entry point include/gsplat_hip.h declares, and the Python surface refuses to
run anywhere but on the GPU (no silent CPU fallback)."""

import os
import re
import subprocess

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gsplat_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(gsplat_hip_\w+)\s*\(", txt)))


def test_header_matches_binding():
    from gsplat_hip import _lib
    assert header_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_symbol():
    from gsplat_hip import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gsplat_hip_\w+)", out))
    missing = set(header_symbols()) - exported
    assert not missing, missing


def test_library_loads_and_abi_version():
    from gsplat_hip import _lib
    lib = _lib.load()
    assert lib.gsplat_hip_abi_version() == _lib.ABI_VERSION
    for d in (1, 2, 3, 4, 8, 16, 32):
        assert lib.gsplat_hip_rasterize_supported_channels(d) == 1
    assert lib.gsplat_hip_rasterize_supported_channels(5) == 0
    # host-only queries (no kernel launch)
    assert lib.gsplat_hip_isect_workspace_bytes(1000) >= 8 * 4


def test_library_is_gfx950():
    from gsplat_hip import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_cpu_tensors_are_refused():
    import gsplat_hip
    from gsplat_hip._lib import GsplatHipError
    means = torch.randn(4, 3)
    with pytest.raises(GsplatHipError):
        gsplat_hip.fully_fused_projection(means, None, torch.randn(4, 4), torch.rand(4, 3),
                                          torch.eye(4)[None], torch.eye(3)[None], 8, 8,
                                          packed=False)


def test_argument_errors_match_reference():
    import gsplat_hip
    C, N = 1, 5
    with pytest.raises(ValueError):  # _wrapper.py:246-248
        gsplat_hip.rasterize_to_pixels(torch.zeros(C, N, 2), torch.zeros(C, N, 3),
                                       torch.zeros(C, N, 0), torch.zeros(C, N), 16, 16, 16,
                                       torch.zeros(C, 1, 1, dtype=torch.int32),
                                       torch.zeros(0, dtype=torch.int32))
    with pytest.raises(NotImplementedError):  # _wrapper.py:322-323
        gsplat_hip.fully_fused_projection(torch.zeros(N, 3), None, torch.zeros(N, 4),
                                          torch.zeros(N, 3), torch.eye(4)[None],
                                          torch.eye(3)[None], 8, 8, camera_model="ortho")
    with pytest.raises(AssertionError):
        gsplat_hip.spherical_harmonics(3, torch.zeros(N, 3), torch.zeros(N, 9, 3))
