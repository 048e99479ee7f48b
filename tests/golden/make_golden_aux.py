"""Golden vectors for quat_scale_to_covar_preci from the REFERENCE's own torch
implementation `_quat_scale_to_covar_preci` (gsplat/cuda/_torch_impl.py:41-71),
the function the reference test compares its CUDA kernel against
(tests/test_basic.py:54-96).  Run in the build container only:

    python tests/golden/make_golden_aux.py

Gradients come from torch autograd with seeded random cotangents.  Only the
produced arrays are committed.
"""

import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    pkg = types.ModuleType("gsplat")
    pkg.__path__ = [os.path.join(REF, "gsplat")]
    sys.modules["gsplat"] = pkg
    from gsplat.cuda._torch_impl import _quat_scale_to_covar_preci

    g = torch.Generator().manual_seed(3)
    N = 500
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.5 + 0.05
    for triu in (False, True):
        q = quats.clone().requires_grad_(True)
        s = scales.clone().requires_grad_(True)
        cov, pre = _quat_scale_to_covar_preci(q, s, triu=triu)
        vc = torch.randn(cov.shape, generator=g)
        vp = torch.randn(pre.shape, generator=g)
        vq, vs = torch.autograd.grad((cov * vc).sum() + (pre * vp).sum(), (q, s))
        np.savez_compressed(os.path.join(OUT, f"covar_preci_triu{int(triu)}.npz"),
                            quats=quats.numpy(), scales=scales.numpy(),
                            covars=cov.detach().numpy(), precis=pre.detach().numpy(),
                            v_covars=vc.numpy(), v_precis=vp.numpy(), v_quats=vq.numpy(),
                            v_scales=vs.numpy())
        print("triu", triu, cov.shape)


if __name__ == "__main__":
    main()
