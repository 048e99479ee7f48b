"""CPU oracle for the auxiliary strategy/optimizer kernels -- TEST
INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

numpy float32 restatements of the reference's CUDA kernels
(hieu1999210/gsplat-triton @ /root/reference):
  covar_preci   gsplat/cuda/csrc/QuatScaleToCovarCUDA.cu (+ Utils.cuh:142-303)
                -- pinned to the reference's own torch implementation
                `_quat_scale_to_covar_preci` (gsplat/cuda/_torch_impl.py:41-71)
                by tests/golden/make_golden_aux.py -> covar_preci_*.npz
  relocation    gsplat/cuda/csrc/RelocationCUDA.cu:10-44 -- parity unpinned
                (no reference fixture; checked by the identity
                1 - (1 - o')^n = o of the MCMC paper, Eq. 8)
  adam          gsplat/cuda/csrc/AdamCUDA.cu:12-46 -- restated update, checked
                against the same formula in torch ops
"""

import math

import numpy as np

f32 = np.float32


def quat_to_R(q):
    q = np.asarray(q, f32)
    q = q / np.sqrt((q * q).sum(-1, keepdims=True))
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)
    return R.reshape(q.shape[:-1] + (3, 3)).astype(f32)


def covar_preci(quats, scales, triu=False):
    """(covars, precis): R S^2 R^T and R S^-2 R^T, [N,3,3] or [N,6]."""
    R = quat_to_R(quats)
    s = np.asarray(scales, f32)
    out = []
    for w in (s * s, 1.0 / (s * s)):
        M = (R * w[:, None, :]) @ np.swapaxes(R, -1, -2)
        if triu:
            M = M.reshape(-1, 9)[:, [0, 1, 2, 4, 5, 8]]
        out.append(M.astype(f32))
    return out[0], out[1]


def relocation(opacities, scales, ratios, binoms):
    """RelocationCUDA.cu:10-44 (ratios already clamped to [1, n_max])."""
    o = np.asarray(opacities, np.float64)
    n = np.asarray(ratios, np.int64)
    b = np.asarray(binoms, np.float64)
    no = 1.0 - np.power(1.0 - o, 1.0 / n)
    denom = np.zeros_like(o)
    for idx in range(o.size):
        acc = 0.0
        for i in range(1, n[idx] + 1):
            for k in range(i):
                acc += b[i - 1, k] * ((-1.0) ** k / math.sqrt(k + 1)) * no[idx] ** (k + 1)
        denom[idx] = acc
    coeff = o / denom
    return no.astype(f32), (np.asarray(scales, np.float64) * coeff[:, None]).astype(f32)


def adam(param, grad, m, v, valid, lr, b1, b2, eps):
    """AdamCUDA.cu:12-46 with a per-row (dim 0) visibility mask; returns new
    (param, m, v)."""
    p, g, m, v = (np.asarray(x, f32).copy() for x in (param, grad, m, v))
    m2 = b1 * m + (1 - b1) * g
    v2 = b2 * v + (1 - b2) * g * g
    p2 = p - lr * m2 / (np.sqrt(v2) + eps)
    if valid is None:
        return p2.astype(f32), m2.astype(f32), v2.astype(f32)
    sel = np.asarray(valid, bool).reshape((-1,) + (1,) * (p.ndim - 1))
    return (np.where(sel, p2, p).astype(f32), np.where(sel, m2, m).astype(f32),
            np.where(sel, v2, v).astype(f32))
