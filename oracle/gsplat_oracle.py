"""CPU oracle for the gsplat hot path -- TEST INFRASTRUCTURE ONLY.

This module is a numpy (float32) restatement of the reference's Triton
backend, `hieu1999210/gsplat-triton` @ /root/reference/gsplat/triton_impl.
It is the *checker*: only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import it.  The product
(`gsplat-triton_amd/gsplat_hip`) never imports, links or calls it.

Pinning: every function is checked against golden vectors produced by running
the reference Triton kernels under TRITON_INTERPRET=1
(`tests/golden/make_golden.py`, `tests/test_oracle_golden.py`).

Semantics followed (reference file:line):
  proj_fwd       fused_projection_fwd.py:16-228 (+ cam_proj.py:5-81,
                 quat_scale_to_covar.py:7-64,147-203, transform.py:7-35,122-181,
                 util_kernels.py:5-24,64-94)
  proj_bwd       fused_projection_bwd.py:24-363 (+ the *_vjp device functions)
  sh_fwd/sh_bwd  sh_fwd.py:69-191, sh_bwd.py:36-380
  isect_tiles    isect_tiles.py:13-282 (Triton tile-bit convention, L1)
  isect_offset   isect_offset.py:8-63 (count(ids < tile) semantics; see L9)
  raster_fwd     rasterize_to_pixels_fwd.py:13-196 (log-space transmittance)
  raster_bwd     rasterize_to_pixels_bwd.py:13-337
"""

import numpy as np

f32 = np.float32  # working precision; `precision(np.float64)` for an exact-math check


def _f(x):
    return np.asarray(x, dtype=f32)


class precision:
    """Run the oracle in another float type, e.g. float64 to measure how far
    an fp32 implementation (the reference's, or the HIP one) is from exact
    arithmetic on long tiles:  `with precision(np.float64): raster_bwd(...)`."""

    def __init__(self, dtype):
        self.dtype = dtype

    def __enter__(self):
        global f32
        self.prev, f32 = f32, self.dtype
        return self

    def __exit__(self, *exc):
        global f32
        f32 = self.prev
        return False


# ------------------------------------------------------------------ helpers
def quat_to_R(q):
    """quat_scale_to_covar.py:147-203 (wxyz, normalised with rsqrt)."""
    q = _f(q)
    q0, q1, q2, q3 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    inv = f32(1.0) / np.sqrt(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3)
    w, x, y, z = q0 * inv, q1 * inv, q2 * inv, q3 * inv
    x2, y2, z2 = x * x, y * y, z * z
    xy, xz, yz = x * y, x * z, y * z
    xw, yw, zw = x * w, y * w, z * w
    R = np.stack([
        1 - 2 * (y2 + z2), 2 * (xy - zw), 2 * (xz + yw),
        2 * (xy + zw), 1 - 2 * (x2 + z2), 2 * (yz - xw),
        2 * (xz - yw), 2 * (yz + xw), 1 - 2 * (x2 + y2),
    ], -1).astype(f32)
    return R.reshape(*R.shape[:-1], 3, 3)


def quat_to_R_vjp(q, dR):
    """quat_scale_to_covar.py:206-271."""
    q = _f(q)
    q0, q1, q2, q3 = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    inv = f32(1.0) / np.sqrt(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3)
    w, x, y, z = q0 * inv, q1 * inv, q2 * inv, q3 * inv
    d = lambda i, j: dR[..., i, j]
    zy_m_yz = d(2, 1) - d(1, 2)
    xz_m_zx = d(0, 2) - d(2, 0)
    yx_m_xy = d(1, 0) - d(0, 1)
    xy_p_yx = d(0, 1) + d(1, 0)
    xz_p_zx = d(0, 2) + d(2, 0)
    yz_p_zy = d(1, 2) + d(2, 1)
    dw = 2 * (x * zy_m_yz + y * xz_m_zx + z * yx_m_xy)
    dx = 2 * (-2 * x * (d(1, 1) + d(2, 2)) + y * xy_p_yx + z * xz_p_zx + w * zy_m_yz)
    dy = 2 * (x * xy_p_yx - 2 * y * (d(0, 0) + d(2, 2)) + z * yz_p_zy + w * xz_m_zx)
    dz = 2 * (x * xz_p_zx + y * yz_p_zy - 2 * z * (d(0, 0) + d(1, 1)) + w * yx_m_xy)
    dot = w * dw + x * dx + y * dy + z * dz
    return np.stack([(dw - w * dot) * inv, (dx - x * dot) * inv,
                     (dy - y * dot) * inv, (dz - z * dot) * inv], -1).astype(f32)


def quat_scale_to_covar(q, s):
    """quat_scale_to_covar.py:7-64: C = (R S)(R S)^T."""
    R = quat_to_R(q)
    RS = R * _f(s)[..., None, :]
    return (RS @ np.swapaxes(RS, -1, -2)).astype(f32)


def quat_scale_to_covar_vjp(q, s, dC):
    """quat_scale_to_covar.py:67-144 (dC treated as symmetric)."""
    R = quat_to_R(q)
    s = _f(s)
    dRS = dC @ (2 * R * s[..., None, :])
    dq = quat_to_R_vjp(q, dRS * s[..., None, :])
    ds = (R * dRS).sum(-2)
    return dq, ds.astype(f32)


# --------------------------------------------------------------- projection
def _persp(mc, cc, fx, fy, cx, cy, W, H, margin=0.15):
    """cam_proj.py:5-81. mc [..,3], cc [..,3,3]; intrinsics broadcastable."""
    x, y, z = mc[..., 0], mc[..., 1], mc[..., 2]
    iz = f32(1.0) / z
    mx = f32(margin) * f32(W) / fx
    my = f32(margin) * f32(H) / fy
    sx_raw, sy_raw = x * iz, y * iz
    sx = np.clip(sx_raw, -mx - cx / fx, mx + (f32(W) - cx) / fx)
    sy = np.clip(sy_raw, -my - cy / fy, my + (f32(H) - cy) / fy)
    Jxx, Jxz = fx * iz, -fx * sx * iz
    Jyy, Jyz = fy * iz, -fy * sy * iz
    c = lambda i, j: cc[..., i, j]
    cxx = Jxx * c(0, 0) * Jxx + 2 * Jxx * c(0, 2) * Jxz + Jxz * c(2, 2) * Jxz
    cxy = Jxx * (c(0, 1) * Jyy + c(0, 2) * Jyz) + Jxz * (c(1, 2) * Jyy + c(2, 2) * Jyz)
    cyy = Jyy * c(1, 1) * Jyy + 2 * Jyy * c(1, 2) * Jyz + Jyz * c(2, 2) * Jyz
    m2 = np.stack([fx * x * iz + cx, fy * y * iz + cy], -1)
    return m2.astype(f32), cxx, cxy, cyy


def _cam(viewmats, Ks):
    vm = _f(viewmats)
    K = _f(Ks)
    R = vm[:, :3, :3]
    t = vm[:, :3, 3]
    fx, fy = K[:, 0, 0][:, None], K[:, 1, 1][:, None]
    cx, cy = K[:, 0, 2][:, None], K[:, 1, 2][:, None]
    return R, t, fx, fy, cx, cy


def proj_fwd(means, quats, scales, viewmats, Ks, W, H, eps2d=0.3, near=0.01,
             far=1e10, radius_clip=0.0, calc_comp=False):
    """fused_projection_fwd.py:16-228 -> radii i32[C,N], means2d[C,N,2],
    depths[C,N], conics[C,N,3], comps[C,N] (or None).

    Entries with radii == 0 are set to 0 (the reference leaves them
    uninitialised, L4)."""
    means, quats, scales = _f(means), _f(quats), _f(scales)
    R, t, fx, fy, cx, cy = _cam(viewmats, Ks)
    c3 = quat_scale_to_covar(quats, scales)                       # [N,3,3]
    mc = np.einsum("cij,nj->cni", R, means).astype(f32) + t[:, None, :]
    cc = np.einsum("cij,njk,clk->cnil", R, c3, R).astype(f32)    # R C R^T
    depths = mc[..., 2].copy()
    keep = (depths > f32(near)) & (depths < f32(far))
    with np.errstate(all="ignore"):
        m2, cxx, cxy, cyy = _persp(mc, cc, fx, fy, cx, cy, W, H)
        det0 = cxx * cyy - cxy * cxy
        cxx = cxx + f32(eps2d)
        cyy = cyy + f32(eps2d)
        det = cxx * cyy - cxy * cxy
        comp = np.sqrt(np.clip(det0 / det, 0.0, np.inf)).astype(f32)
        keep &= det > 0
        inv = f32(1.0) / det
        conics = np.stack([inv * cyy, -inv * cxy, inv * cxx], -1).astype(f32)
        b = f32(0.5) * (cxx + cyy)
        v1 = b + np.sqrt(np.maximum(f32(0.01), b * b - det))
        r = np.ceil(f32(3.0) * np.sqrt(v1)).astype(f32)
        keep &= (r > f32(radius_clip)) & (m2[..., 0] + r > 0) & (m2[..., 0] - r < W) \
            & (m2[..., 1] + r > 0) & (m2[..., 1] - r < H)
    radii = np.where(keep, r, 0).astype(np.int32)
    m2 = np.where(keep[..., None], m2, 0).astype(f32)
    conics = np.where(keep[..., None], conics, 0).astype(f32)
    comp = np.where(keep, comp, 0).astype(f32) if calc_comp else None
    return radii, m2, depths.astype(f32), conics, comp


def proj_bwd(means, quats, scales, viewmats, Ks, W, H, eps2d, radii, conics, comps,
             v_means2d, v_depths, v_conics, v_comps, viewmats_requires_grad=True):
    """fused_projection_bwd.py:24-363. Returns v_means[N,3], v_quats[N,4],
    v_scales[N,3], v_viewmats[C,4,4] (None if not requested).  Only entries
    with radii > 0 contribute (fused_projection_bwd.py:68-69)."""
    means, quats, scales = _f(means), _f(quats), _f(scales)
    R, t, fx, fy, cx, cy = _cam(viewmats, Ks)
    C, N = radii.shape
    valid = radii > 0
    ci, ni = np.nonzero(valid)
    v_means = np.zeros((N, 3), f32)
    v_quats = np.zeros((N, 4), f32)
    v_scales = np.zeros((N, 3), f32)
    v_vm = np.zeros((C, 4, 4), f32)
    if len(ci) == 0:
        return v_means, v_quats, v_scales, (v_vm if viewmats_requires_grad else None)
    cn = _f(conics)[ci, ni]
    a, b, c = cn[:, 0], cn[:, 1], cn[:, 2]
    vc = _f(v_conics)[ci, ni]
    va, vb, vcc = vc[:, 0], vc[:, 1] * f32(0.5), vc[:, 2]
    # util_kernels.py:27-61 inverse vjp
    dxx = -(a * va * a + b * vcc * b + 2 * b * vb * a)
    dxy = -(a * vb * c + b * vb * b + b * vcc * c + a * va * b)
    dyy = -(b * va * b + c * vcc * c + 2 * c * vb * b)
    if comps is not None:
        cp = _f(comps)[ci, ni]
        vcp = _f(v_comps)[ci, ni]
        det_i = a * c - b * b
        Da = f32(0.5) * vcp / (cp + f32(1e-6))
        oma = 1 - cp * cp
        dxx = dxx + Da * (oma * a - f32(eps2d) * det_i)
        dxy = dxy + Da * (oma * b)
        dyy = dyy + Da * (oma * c - f32(eps2d) * det_i)
    m = means[ni]
    q = quats[ni]
    s = scales[ni]
    Rc = R[ci]
    c3 = quat_scale_to_covar(q, s)
    cc = (Rc @ c3 @ np.swapaxes(Rc, -1, -2)).astype(f32)
    mc = np.einsum("kij,kj->ki", Rc, m).astype(f32) + t[ci]
    fxk, fyk, cxk, cyk = fx[ci, 0], fy[ci, 0], cx[ci, 0], cy[ci, 0]
    x, y, z = mc[:, 0], mc[:, 1], mc[:, 2]
    iz = f32(1.0) / z
    mx = f32(0.15) * f32(W) / fxk
    my = f32(0.15) * f32(H) / fyk
    sx, sy = x * iz, y * iz
    lox, hix = -mx - cxk / fxk, mx + (f32(W) - cxk) / fxk
    loy, hiy = -my - cyk / fyk, my + (f32(H) - cyk) / fyk
    clx = (sx < lox) | (sx > hix)
    cly = (sy < loy) | (sy > hiy)
    sx, sy = np.clip(sx, lox, hix), np.clip(sy, loy, hiy)
    Jxx, Jxz = fxk * iz, -fxk * sx * iz
    Jyy, Jyz = fyk * iz, -fyk * sy * iz
    # cam_proj.py:161-168
    v3 = np.zeros((len(ci), 3, 3), f32)
    v3[:, 0, 0] = Jxx * dxx * Jxx
    v3[:, 1, 1] = Jyy * dyy * Jyy
    v3[:, 2, 2] = Jxz * dxx * Jxz + Jyz * dyy * Jyz + 2 * Jyz * dxy * Jxz
    v3[:, 0, 1] = v3[:, 1, 0] = Jxx * dxy * Jyy
    v3[:, 0, 2] = v3[:, 2, 0] = Jxx * dxx * Jxz + Jxx * dxy * Jyz
    v3[:, 1, 2] = v3[:, 2, 1] = Jyy * dxy * Jxz + Jyy * dyy * Jyz
    vm2 = _f(v_means2d)[ci, ni]
    vmx = Jxx * vm2[:, 0]
    vmy = Jyy * vm2[:, 1]
    vmz = Jxz * vm2[:, 0] + Jyz * vm2[:, 1]
    c_ = lambda i, j: cc[:, i, j]
    Jc_xx = Jxx * c_(0, 0) + Jxz * c_(0, 2)
    Jc_xy = Jxx * c_(0, 1) + Jxz * c_(1, 2)
    Jc_xz = Jxx * c_(0, 2) + Jxz * c_(2, 2)
    Jc_yx = Jyy * c_(0, 1) + Jyz * c_(0, 2)
    Jc_yy = Jyy * c_(1, 1) + Jyz * c_(1, 2)
    Jc_yz = Jyy * c_(1, 2) + Jyz * c_(2, 2)
    vJxx = 2 * (dxx * Jc_xx + dxy * Jc_yx)
    vJxz = 2 * (dxx * Jc_xz + dxy * Jc_yz)
    vJyy = 2 * (dxy * Jc_xy + dyy * Jc_yy)
    vJyz = 2 * (dxy * Jc_xz + dyy * Jc_yz)
    iz2 = iz * iz
    vmx = vmx + np.where(clx, 0, -vJxz * fxk * iz2)
    vmy = vmy + np.where(cly, 0, -vJyz * fyk * iz2)
    tmp = vJxx * Jxx + vJyy * Jyy + 2 * (vJxz * Jxz + vJyz * Jyz)
    tmp = tmp - np.where(clx, vJxz * Jxz, 0) - np.where(cly, vJyz * Jyz, 0)
    vmz = vmz - iz * tmp
    vmz = vmz + _f(v_depths)[ci, ni]
    vmc = np.stack([vmx, vmy, vmz], -1).astype(f32)
    # transform.py:38-119: v_m = R^T v_mc; v_T = v_mc; v_R = v_mc m^T
    vmw = np.einsum("kji,kj->ki", Rc, vmc).astype(f32)
    np.add.at(v_means, ni, vmw)
    # transform.py:184-297: v_c3 = R^T v3 R; v_R += 2 v3 R c3
    vSR = v3 @ Rc
    vc3 = (np.swapaxes(Rc, -1, -2) @ vSR).astype(f32)
    if viewmats_requires_grad:
        vR = vmc[:, :, None] * m[:, None, :] + 2 * vSR @ c3
        for k in range(3):
            np.add.at(v_vm[:, k, 3], ci, vmc[:, k])
            for l in range(3):
                np.add.at(v_vm[:, k, l], ci, vR[:, k, l])
    dq, ds = quat_scale_to_covar_vjp(q, s, vc3)
    np.add.at(v_quats, ni, dq)
    np.add.at(v_scales, ni, ds)
    return v_means, v_quats, v_scales, (v_vm if viewmats_requires_grad else None)


# ------------------------------------------------------ spherical harmonics
def _sh_basis(deg, d):
    """Returns normalised (x,y,z), inorm and the list of basis values
    (sh_fwd.py:88-189 / sh_bwd.py:60-330 constants)."""
    x, y, z = d[..., 0], d[..., 1], d[..., 2]
    inorm = f32(1.0) / np.sqrt(x * x + y * y + z * z)
    x, y, z = x * inorm, y * inorm, z * inorm
    B = [np.full_like(x, f32(0.28209479177387814))]
    if deg >= 1:
        B += [f32(-0.4886025119029199) * y, f32(0.4886025119029199) * z,
              f32(-0.4886025119029199) * x]
    if deg >= 2:
        zz = z * z
        g2, h2 = 2 * x * y, x * x - y * y
        c21 = f32(-1.0925484305920792) * z
        B += [f32(0.5462742152960396) * g2, c21 * y,
              f32(0.9461746957575601) * zz - f32(0.3153915652525201), c21 * x,
              f32(0.5462742152960396) * h2]
    if deg >= 3:
        g3, h3 = x * g2 + y * h2, x * h2 - y * g2
        c31 = f32(-2.285228997322329) * zz + f32(0.4570457994644658)
        B += [f32(-0.5900435899266435) * g3, f32(1.445305721320277) * g2 * z, c31 * y,
              z * (f32(1.865881662950577) * zz - f32(1.119528997770346)), c31 * x,
              f32(1.445305721320277) * h2 * z, f32(-0.5900435899266435) * h3]
    if deg >= 4:
        g4, h4 = x * g3 + y * h3, x * h3 - y * g3
        c41 = z * (f32(-4.683325804901024) * zz + f32(2.0071396306718676))
        c42 = f32(3.31161143515146) * zz - f32(0.47308734787878)
        B += [f32(0.6258357354491761) * g4, f32(-1.7701307697799304) * g3 * z, c42 * g2,
              c41 * y,
              zz * (f32(3.7024941420321507) * zz - f32(3.1735664074561294)) + f32(0.31735664074561293),
              c41 * x, c42 * h2, f32(-1.7701307697799304) * h3 * z,
              f32(0.6258357354491761) * h4]
    return (x, y, z), inorm, B


def sh_fwd(deg, dirs, coeffs, masks=None):
    """sh_fwd.py:69-233 (+ _wrapper.py:567-568 mask zeroing)."""
    dirs, coeffs = _f(dirs), _f(coeffs)
    with np.errstate(all="ignore"):
        _, _, B = _sh_basis(deg, dirs)
    out = np.zeros(coeffs.shape[:-2] + (coeffs.shape[-1],), f32)
    for k, b in enumerate(B):
        out += b[..., None] * coeffs[..., k, :]
    if masks is not None:
        out[~masks] = 0
    return out


def sh_bwd(deg, dirs, coeffs, v_colors, masks=None, compute_v_dirs=True):
    """sh_bwd.py:36-436: v_coeffs (first (d+1)^2 bases, rest 0) and v_dirs
    through the normalisation (sh_bwd.py:367-380)."""
    dirs, coeffs, v_colors = _f(dirs), _f(coeffs), _f(v_colors)
    with np.errstate(all="ignore"):
        (x, y, z), inorm, B = _sh_basis(deg, dirs)
    v_coeffs = np.zeros_like(coeffs)
    for k, b in enumerate(B):
        v_coeffs[..., k, :] = b[..., None] * v_colors
    v_dirs = None
    if compute_v_dirs:
        sh = lambda k: coeffs[..., k, :]
        vx = vy = vz = 0
        if deg >= 1:
            vy = f32(-0.4886025119029199) * sh(1)
            vz = f32(0.4886025119029199) * sh(2)
            vx = f32(-0.4886025119029199) * sh(3)
            x_, y_, z_ = x[..., None], y[..., None], z[..., None]
        if deg >= 2:
            zz, xz, yz = z_ * z_, x_ * z_, y_ * z_
            g2, h2 = 2 * x_ * y_, x_ * x_ - y_ * y_
            c21 = f32(-1.0925484305920792) * z_
            c22g = f32(1.0925484305920792) * y_
            c22h = f32(1.0925484305920792) * x_
            vx = vx + c22g * sh(4) + c21 * sh(7) + c22h * sh(8)
            vy = vy + c22h * sh(4) + c21 * sh(5) - c22g * sh(8)
            vz = vz - c22g * sh(5) + f32(1.8923493915151202) * z_ * sh(6) - c22h * sh(7)
        if deg >= 3:
            g3, h3 = x_ * g2 + y_ * h2, x_ * h2 - y_ * g2
            c31 = f32(-2.2852289973223288) * zz + f32(0.4570457994644658)
            a3g = f32(-1.7701307697799304) * g2
            a3h = f32(-1.7701307697799304) * h2
            b3y = f32(2.890611442640554) * yz
            b3x = f32(2.890611442640554) * xz
            vx = vx + a3g * sh(9) + b3y * sh(10) + c31 * sh(13) + b3x * sh(14) + a3h * sh(15)
            vy = vy + a3h * sh(9) + b3x * sh(10) + c31 * sh(11) - b3y * sh(14) - a3g * sh(15)
            vz = vz + (f32(1.445305721320277) * g2 * sh(10) - f32(4.570457994644658) * yz * sh(11)
                       - f32(2.449489742783178) * c31 * sh(12)
                       - f32(4.570457994644658) * xz * sh(13) + f32(1.445305721320277) * h2 * sh(14))
        if deg >= 4:
            c41 = z_ * (f32(-4.683325804901024) * zz + f32(2.0071396306718676))
            c42 = f32(3.31161143515146) * zz - f32(0.47308734787878)
            a4g = f32(2.5033429417967046) * g3
            a4h = f32(2.5033429417967046) * h3
            b4g = f32(-5.310392309339791) * g2 * z_
            b4h = f32(-5.310392309339791) * h2 * z_
            c4g = c42 * 2 * y_
            c4h = c42 * 2 * x_
            vx = vx + (a4g * sh(16) + b4g * sh(17) + c4g * sh(18) + c41 * sh(21)
                       + c4h * sh(22) + b4h * sh(23) + a4h * sh(24))
            vy = vy + (a4h * sh(16) + b4h * sh(17) + c4h * sh(18) + c41 * sh(19)
                       - c4g * sh(22) - b4g * sh(23) - a4g * sh(24))
            vz = vz + (f32(-1.7701307697799304) * g3 * sh(17)
                       - f32(1.2472191289246473) * b4g * sh(18)
                       - f32(2.1213203435596424) * c4g * sh(19)
                       - f32(3.162277660168379) * c41 * sh(20)
                       - f32(2.1213203435596424) * c4h * sh(21)
                       - f32(1.2472191289246473) * b4h * sh(22)
                       - f32(1.7701307697799304) * h3 * sh(23))
        if deg >= 1:
            # per colour channel lane, then atomically summed over channels
            vx, vy, vz = vx * v_colors, vy * v_colors, vz * v_colors
            dot = x_ * vx + y_ * vy + z_ * vz
            iv = inorm[..., None]
            v_dirs = np.stack([((vx - dot * x_) * iv).sum(-1), ((vy - dot * y_) * iv).sum(-1),
                               ((vz - dot * z_) * iv).sum(-1)], -1).astype(f32)
        else:
            v_dirs = np.zeros_like(dirs)
    if masks is not None:
        v_coeffs[~masks] = 0
        if v_dirs is not None:
            v_dirs[~masks] = 0
    return v_coeffs, v_dirs


# ------------------------------------------------------------------- isect
def tile_rect(means2d, radii, ts, tw, th):
    """isect_tiles.py:255-282: float32 floor/ceil of (p -/+ r)/ts, clamped."""
    p = _f(means2d)
    r = _f(radii)
    t = f32(ts)
    with np.errstate(all="ignore"):
        xmin = np.clip(np.floor((p[..., 0] - r) / t), 0, tw).astype(np.int64)
        xmax = np.clip(np.ceil((p[..., 0] + r) / t), 0, tw).astype(np.int64)
        ymin = np.clip(np.floor((p[..., 1] - r) / t), 0, th).astype(np.int64)
        ymax = np.clip(np.ceil((p[..., 1] + r) / t), 0, th).astype(np.int64)
    return xmin, xmax, ymin, ymax


def tile_bits(n):
    return int(n - 1).bit_length() if n > 0 else 0


def isect_tiles(means2d, radii, depths, ts, tw, th, sort=True):
    """isect_tiles.py:13-131. Returns tiles_per_gauss i32[C,N],
    isect_ids i64[n], flatten_ids i32[n] (stable sort on the id bits)."""
    C, N = radii.shape
    xmin, xmax, ymin, ymax = tile_rect(means2d, radii, ts, tw, th)
    tpg = np.where(radii > 0, (xmax - xmin) * (ymax - ymin), 0).astype(np.int32)
    flat_tpg = tpg.reshape(-1).astype(np.int64)
    n = int(flat_tpg.sum())
    tb = tile_bits(tw * th)
    dbits = _f(depths).reshape(-1).view(np.int32).astype(np.int64)  # sign-extended
    gid = np.repeat(np.arange(C * N, dtype=np.int64), flat_tpg)
    start = np.cumsum(flat_tpg) - flat_tpg
    local = np.arange(n, dtype=np.int64) - np.repeat(start, flat_tpg)
    xm, ym = xmin.reshape(-1)[gid], ymin.reshape(-1)[gid]
    xs = (xmax - xmin).reshape(-1)[gid]
    tx = xm + local % np.maximum(xs, 1)
    ty = ym + local // np.maximum(xs, 1)
    tile = ty * tw + tx
    cam = gid // N if N > 0 else gid
    ids = (cam << (tb + 32)) | (tile << 32) | dbits[gid]
    fids = gid.astype(np.int32)
    if sort and n:
        nbits = 32 + tb + tile_bits(C)
        key = ids & ((1 << nbits) - 1) if nbits < 63 else ids
        order = np.argsort(key, kind="stable")
        ids, fids = ids[order], fids[order]
    return tpg, ids, fids


def isect_offset_encode(isect_ids, C, tw, th):
    """offsets[c, ty, tx] = #isects whose (cam, tile) key < (c, tile)
    (isect_offset.py:39-63; CUDA semantics for the n_isects == 1 corner, L9)."""
    n_tiles = tw * th
    tb = tile_bits(n_tiles)
    ids = np.asarray(isect_ids, np.int64) >> 32
    key = (ids >> tb) * n_tiles + (ids & ((1 << tb) - 1))
    off = np.searchsorted(key, np.arange(C * n_tiles), side="left").astype(np.int32)
    return off.reshape(C, th, tw)


# ------------------------------------------------------------ rasterization
def _tile_ranges(offsets, n_isects):
    flat = np.asarray(offsets, np.int64).reshape(-1)
    ends = np.append(flat[1:], n_isects)
    return flat, ends


def raster_fwd(means2d, conics, colors, opacities, backgrounds, W, H, ts, offsets,
               flatten_ids, tiles=None):
    """rasterize_to_pixels_fwd.py:13-196 (log-space T, exclusive stop at
    log T <= log(1e-4)).  Returns colors[C,H,W,D], alphas[C,H,W,1],
    last_ids i32[C,H,W].  `tiles`: optional iterable of flat tile indices to
    render (bounded CPU-baseline sample); other pixels stay 0."""
    C, th, tw = offsets.shape
    D = colors.shape[-1]
    m2 = _f(means2d).reshape(-1, 2)
    cn = _f(conics).reshape(-1, 3)
    cl = _f(colors).reshape(-1, D)
    op = _f(opacities).reshape(-1)
    fids = np.asarray(flatten_ids, np.int64)
    starts, ends = _tile_ranges(offsets, len(fids))
    out_c = np.zeros((C, H, W, D), f32)
    out_a = np.zeros((C, H, W, 1), f32)
    out_l = np.zeros((C, H, W), np.int32)
    ly, lx = np.meshgrid(np.arange(ts), np.arange(ts), indexing="ij")
    for t in (range(C * th * tw) if tiles is None else tiles):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        y0, x0 = ty * ts, tx * ts
        pyi, pxi = (ly + y0).reshape(-1), (lx + x0).reshape(-1)
        inside = (pyi < H) & (pxi < W)
        px, py = pxi.astype(f32) + f32(0.5), pyi.astype(f32) + f32(0.5)
        s, e = starts[t], ends[t]
        logT = np.zeros(ts * ts, f32)
        acc = np.zeros((ts * ts, D), f32)
        last = np.zeros(ts * ts, np.int32)
        if e > s:
            g = fids[s:e]
            dx = m2[g, 0][:, None] - px[None]
            dy = m2[g, 1][:, None] - py[None]
            a, b, cc = cn[g, 0][:, None], cn[g, 1][:, None], cn[g, 2][:, None]
            with np.errstate(all="ignore"):
                sig = f32(0.5) * (a * dx * dx + cc * dy * dy) + b * dx * dy
                al = np.clip(op[g][:, None] * np.exp(-sig), 0, f32(0.999))
                skip = (al < f32(1.0 / 255.0)) | (sig < 0) | ~inside[None]
                al = np.where(skip, 0, al).astype(f32)
                l1 = np.log(f32(1.0) - al)
                lT = np.cumsum(l1, axis=0, dtype=f32)
                skip |= lT <= f32(-9.21034)
                vis = np.where(skip, 0, np.exp(lT - l1) * al).astype(f32)
            acc = (vis[:, :, None] * cl[g][:, None, :]).sum(0, dtype=f32)
            logT = np.where(skip, 0, l1).sum(0, dtype=f32)
            keep = ~skip
            anyk = keep.any(0)
            lastk = (len(g) - 1) - np.argmax(keep[::-1], axis=0)
            last = np.where(anyk, s + lastk, 0).astype(np.int32)
        alpha = f32(1.0) - np.exp(logT)
        if backgrounds is not None:
            acc = acc + (f32(1.0) - alpha)[:, None] * _f(backgrounds)[c][None]
        sel = inside
        out_c[c, pyi[sel], pxi[sel]] = acc[sel]
        out_a[c, pyi[sel], pxi[sel], 0] = alpha[sel]
        out_l[c, pyi[sel], pxi[sel]] = last[sel]
    return out_c, out_a, out_l


def raster_bwd(means2d, conics, colors, opacities, backgrounds, W, H, ts, offsets,
               flatten_ids, render_alphas, last_ids, v_render_colors,
               v_render_alphas, absgrad=False, tiles=None):
    """rasterize_to_pixels_bwd.py:13-337.  Returns v_means2d, v_conics,
    v_colors, v_opacities, v_backgrounds (None without backgrounds),
    v_means2d_abs (None unless absgrad)."""
    C, th, tw = offsets.shape
    D = colors.shape[-1]
    shp2 = means2d.shape
    m2 = _f(means2d).reshape(-1, 2)
    cn = _f(conics).reshape(-1, 3)
    cl = _f(colors).reshape(-1, D)
    op = _f(opacities).reshape(-1)
    G = op.shape[0]
    fids = np.asarray(flatten_ids, np.int64)
    starts, ends = _tile_ranges(offsets, len(fids))
    vm = np.zeros((G, 2), f32)
    vm_abs = np.zeros((G, 2), f32)
    vc = np.zeros((G, 3), f32)
    vcol = np.zeros((G, D), f32)
    vop = np.zeros(G, f32)
    ra = _f(render_alphas)
    vrc = _f(v_render_colors)
    vra = _f(v_render_alphas)
    bg = None if backgrounds is None else _f(backgrounds)
    ly, lx = np.meshgrid(np.arange(ts), np.arange(ts), indexing="ij")
    for t in (range(C * th * tw) if tiles is None else tiles):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        pyi, pxi = (ly + ty * ts).reshape(-1), (lx + tx * ts).reshape(-1)
        inside = (pyi < H) & (pxi < W)
        yc, xc = np.minimum(pyi, H - 1), np.minimum(pxi, W - 1)
        lid = np.where(inside, last_ids[c, yc, xc], 0)
        s = starts[t]
        e = min(ends[t], int(lid.max()) + 1)
        if e <= s:
            continue
        px, py = pxi.astype(f32) + f32(0.5), pyi.astype(f32) + f32(0.5)
        Dra = np.where(inside, vra[c, yc, xc, 0], 0).astype(f32)
        Drc = np.where(inside[:, None], vrc[c, yc, xc], 0).astype(f32)
        Tf = f32(1.0) - np.where(inside, ra[c, yc, xc, 0], 0).astype(f32)
        g = fids[s:e]
        idx = np.arange(s, e)
        dx = m2[g, 0][:, None] - px[None]
        dy = m2[g, 1][:, None] - py[None]
        a, b, cc = cn[g, 0][:, None], cn[g, 1][:, None], cn[g, 2][:, None]
        with np.errstate(all="ignore"):
            sig = f32(0.5) * a * dx * dx + f32(0.5) * cc * dy * dy + b * dx * dy
            ex = np.exp(-sig).astype(f32)
            al = op[g][:, None] * ex
            skip = (idx[:, None] > lid[None]) | (al < f32(1.0 / 255.0)) | (sig < 0)
            al = np.where(skip, 0, al).astype(f32)
            dskip = (al > f32(0.999)) | skip
            al = np.clip(al, 0, f32(0.999))
            l1 = np.log(f32(1.0) - al).astype(f32)
            # exclusive T: log T_final - (inclusive suffix sum of l1)
            suf = np.cumsum(l1[::-1], axis=0, dtype=f32)[::-1]
            T = np.exp(np.log(Tf)[None] - suf).astype(f32)
            gc = cl[g]
            gD = (Drc[None] * gc[:, None, :]).sum(-1, dtype=f32)
            w = T * al
            vcol_t = (w[:, :, None] * Drc[None]).sum(1, dtype=f32)
            r = gD * w
            rD = np.cumsum(r[::-1], axis=0, dtype=f32)[::-1]
            ra_inv = np.exp(-l1)
            Da = ra_inv * (Tf[None] * Dra[None] + T * gD - rD)
            if bg is not None:
                bt = (bg[c][None] * Drc).sum(-1, dtype=f32) * Tf
                Da = Da - ra_inv * bt[None]
            Da = np.where(dskip, 0, Da).astype(f32)
            aD = al * Da
            dmx = -aD * (a * dx + b * dy)
            dmy = -aD * (b * dx + cc * dy)
        np.add.at(vcol, g, vcol_t)
        np.add.at(vop, g, (Da * ex).sum(1, dtype=f32))
        np.add.at(vm, g, np.stack([dmx.sum(1, dtype=f32), dmy.sum(1, dtype=f32)], -1))
        if absgrad:
            np.add.at(vm_abs, g, np.stack([np.abs(dmx).sum(1, dtype=f32),
                                           np.abs(dmy).sum(1, dtype=f32)], -1))
        np.add.at(vc, g, np.stack([(f32(-0.5) * aD * dx * dx).sum(1, dtype=f32),
                                   (-aD * dx * dy).sum(1, dtype=f32),
                                   (f32(-0.5) * aD * dy * dy).sum(1, dtype=f32)], -1))
    v_bg = None
    if bg is not None:  # _wrapper.py:159-162
        v_bg = (vrc * (f32(1.0) - ra)).sum((1, 2), dtype=f32)
    return (vm.reshape(shp2), vc.reshape(conics.shape), vcol.reshape(colors.shape),
            vop.reshape(opacities.shape), v_bg,
            vm_abs.reshape(shp2) if absgrad else None)
