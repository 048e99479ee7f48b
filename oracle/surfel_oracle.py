"""CPU oracle for the 2DGS (surfel) path -- TEST INFRASTRUCTURE ONLY.

A numpy (float32) restatement of the reference's CUDA 2DGS kernels
(hieu1999210/gsplat-triton @ /root/reference/gsplat/cuda/csrc).  Only
`tests/` (and bench's CPU-baseline leg) may import it; the product
(`gsplat-triton_amd/gsplat_hip`) never does.

Semantics followed (reference file:line):
  proj2dgs_fwd    Projection2DGSFused.cu:17-238
  proj2dgs_bwd    Projection2DGSFused.cu:319-457, Projection2DGS.cuh:10-87
                  (quat_to_rotmat_vjp: gsplat/cuda/include/Utils.cuh:166-189)
  raster2dgs_fwd  RasterizeToPixels2DGSFwd.cu:18-452
  raster2dgs_bwd  RasterizeToPixels2DGSBwd.cu:16-700 (+ v_backgrounds of
                  gsplat/cuda/_wrapper.py:1953-1958)

Pinning:
  * projection forward and backward: against the reference's own torch
    implementation `_fully_fused_projection_2dgs`
    (gsplat/cuda/_torch_impl_2dgs.py:9-88) run in this container on the
    reference test's scene and on random scenes (tests/golden/make_golden_2dgs.py
    -> tests/golden/proj2dgs_*.npz), at the reference test's tolerances
    (tests/test_2dgs.py:77-122).
  * rasterization: PARITY UNPINNED against reference outputs -- the
    reference's only CPU rasterizer for 2DGS (`_rasterize_to_pixels_2dgs`,
    _torch_impl_2dgs.py:179-272) needs the CUDA extension
    (`rasterize_to_indices_in_range_2dgs`) and nerfacc, neither of which runs
    here, and the repository ships no 2DGS render fixtures.  The forward is a
    line-by-line restatement; the backward is checked against torch autograd
    of an independent torch restatement of the forward (tests/test_surfel_oracle.py).

Deliberate, documented deviations (same as the HIP path):
  * culled projection entries are zeros (the reference leaves them
    uninitialised; a degenerate AABB returns before writing radii);
  * v_densify is formed from the final v_ray_transforms sums (the reference
    writes it racily from partial sums, RasterizeToPixels2DGSBwd.cu:689-697);
  * masked tiles: alphas / normals / distortion / median / ids are written as
    empty (the reference writes only the background colour).
"""

import numpy as np

f32 = np.float32
ALPHA_MIN = f32(1.0 / 255.0)
ALPHA_MAX = f32(0.999)
T_MIN = f32(1e-4)
FILTER_INV_SQUARE = f32(2.0)


def _f(x):
    return np.asarray(x, dtype=f32)


def quat_to_R(q):
    """Utils.cuh:142-164 (normalised), row-major math matrix [..., 3, 3]."""
    q = _f(q)
    q = q / np.sqrt((q * q).sum(-1, keepdims=True, dtype=f32))
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)
    return R.reshape(q.shape[:-1] + (3, 3)).astype(f32)


def quat_to_R_vjp(q, dR):
    """Utils.cuh:166-189 with dR as the row-major math gradient."""
    q = _f(q)
    inv = f32(1.0) / np.sqrt((q * q).sum(-1, dtype=f32))
    w, x, y, z = (q[..., i] * inv for i in range(4))
    d = dR
    dw = 2 * (x * (d[..., 2, 1] - d[..., 1, 2]) + y * (d[..., 0, 2] - d[..., 2, 0]) +
              z * (d[..., 1, 0] - d[..., 0, 1]))
    dx = 2 * (-2 * x * (d[..., 1, 1] + d[..., 2, 2]) + y * (d[..., 1, 0] + d[..., 0, 1]) +
              z * (d[..., 2, 0] + d[..., 0, 2]) + w * (d[..., 2, 1] - d[..., 1, 2]))
    dy = 2 * (x * (d[..., 1, 0] + d[..., 0, 1]) - 2 * y * (d[..., 0, 0] + d[..., 2, 2]) +
              z * (d[..., 2, 1] + d[..., 1, 2]) + w * (d[..., 0, 2] - d[..., 2, 0]))
    dz = 2 * (x * (d[..., 2, 0] + d[..., 0, 2]) + y * (d[..., 2, 1] + d[..., 1, 2]) -
              2 * z * (d[..., 0, 0] + d[..., 1, 1]) + w * (d[..., 1, 0] - d[..., 0, 1]))
    vn = np.stack([dw, dx, dy, dz], -1).astype(f32)
    qn = np.stack([w, x, y, z], -1)
    return ((vn - (vn * qn).sum(-1, keepdims=True) * qn) * inv[..., None]).astype(f32)


def _frame(means, quats, scales, viewmats):
    R = _f(viewmats)[:, :3, :3]
    t = _f(viewmats)[:, :3, 3]
    mc = np.einsum("cij,nj->cni", R, _f(means)) + t[:, None]
    Rq = quat_to_R(quats)  # [N,3,3]
    RRq = np.einsum("cij,njk->cnik", R, Rq)  # [C,N,3,3]
    s = _f(scales)
    t0 = RRq[..., 0] * s[None, :, 0:1]
    t1 = RRq[..., 1] * s[None, :, 1:2]
    nz = RRq[..., 2]
    return R, mc.astype(f32), t0.astype(f32), t1.astype(f32), nz.astype(f32), Rq


def proj2dgs_fwd(means, quats, scales, viewmats, Ks, W, H, near=0.01, far=1e10, radius_clip=0.0):
    """Projection2DGSFused.cu:17-238.  Returns radii i32[C,N], means2d[C,N,2],
    depths[C,N], ray_transforms[C,N,3,3] (rows of K [t_u | t_v | mean_c]),
    normals[C,N,3]."""
    R, mc, t0, t1, nz, _ = _frame(means, quats, scales, viewmats)
    K = _f(Ks)
    fx, cx, fy, cy = (K[:, 0, 0][:, None], K[:, 0, 2][:, None], K[:, 1, 1][:, None],
                      K[:, 1, 2][:, None])
    M = np.stack([
        fx * t0[..., 0] + cx * t0[..., 2], fx * t1[..., 0] + cx * t1[..., 2],
        fx * mc[..., 0] + cx * mc[..., 2],
        fy * t0[..., 1] + cy * t0[..., 2], fy * t1[..., 1] + cy * t1[..., 2],
        fy * mc[..., 1] + cy * mc[..., 2],
        t0[..., 2], t1[..., 2], mc[..., 2]], -1).astype(f32)  # [C,N,9]
    with np.errstate(all="ignore"):
        dist = M[..., 6] ** 2 + M[..., 7] ** 2 - M[..., 8] ** 2
        fi = f32(1.0) / dist
        mx = fi * M[..., 0] * M[..., 6] + fi * M[..., 1] * M[..., 7] - fi * M[..., 2] * M[..., 8]
        my = fi * M[..., 3] * M[..., 6] + fi * M[..., 4] * M[..., 7] - fi * M[..., 5] * M[..., 8]
        ex = mx * mx - (fi * M[..., 0] ** 2 + fi * M[..., 1] ** 2 - fi * M[..., 2] ** 2)
        ey = my * my - (fi * M[..., 3] ** 2 + fi * M[..., 4] ** 2 - fi * M[..., 5] ** 2)
        radius = np.ceil(f32(3.0) * np.sqrt(np.maximum(f32(1e-4), np.maximum(ex, ey))))
        keep = ~((mc[..., 2] < near) | (mc[..., 2] > far)) & (dist != 0)
        keep &= radius > radius_clip
        keep &= ~((mx + radius <= 0) | (mx - radius >= W) | (my + radius <= 0) |
                  (my - radius >= H))
    sgn = np.where(-(nz * mc).sum(-1) > 0, f32(1.0), f32(-1.0))
    radii = np.where(keep, radius, 0).astype(np.int32)
    means2d = np.where(keep[..., None], np.stack([mx, my], -1), 0).astype(f32)
    rt = np.where(keep[..., None], M, 0).astype(f32).reshape(M.shape[:2] + (3, 3))
    normals = np.where(keep[..., None], nz * sgn[..., None], 0).astype(f32)
    return radii, means2d, mc[..., 2].astype(f32), rt, normals


def proj2dgs_bwd(means, quats, scales, viewmats, Ks, radii, ray_transforms, v_means2d, v_depths,
                 v_normals, v_ray_transforms):
    """Projection2DGSFused.cu:319-457 (+ Projection2DGS.cuh:10-87).  Returns
    v_means[N,3], v_quats[N,4], v_scales[N,3] (v_scales[:,2] = 0)."""
    R, mc, t0, t1, nz, Rq = _frame(means, quats, scales, viewmats)
    C, N = mc.shape[:2]
    K = _f(Ks)
    r = _f(ray_transforms).reshape(C, N, 9)
    V = _f(v_ray_transforms).reshape(C, N, 9).copy()
    if v_depths is not None:
        V[..., 8] += _f(v_depths)
    gx, gy = _f(v_means2d)[..., 0], _f(v_means2d)[..., 1]
    with np.errstate(all="ignore"):
        fi = f32(1.0) / (r[..., 6] ** 2 + r[..., 7] ** 2 - r[..., 8] ** 2)
        f2 = f32(2.0) * fi * fi
        e6, e7, e8 = fi - f2 * r[..., 6] ** 2, fi - f2 * r[..., 7] ** 2, fi + f2 * r[..., 8] ** 2
        add = np.stack([gx * fi * r[..., 6], gx * fi * r[..., 7], -gx * fi * r[..., 8],
                        gy * fi * r[..., 6], gy * fi * r[..., 7], -gy * fi * r[..., 8],
                        gx * r[..., 0] * e6 + gy * r[..., 3] * e6,
                        gx * r[..., 1] * e7 + gy * r[..., 4] * e7,
                        -gx * r[..., 2] * e8 - gy * r[..., 5] * e8], -1)
    has = ((gx != 0) | (gy != 0))[..., None]
    V = np.where(has, V + np.nan_to_num(add), V).astype(f32)
    Vm = V.reshape(C, N, 3, 3)
    fx, cx, fy, cy = K[:, 0, 0], K[:, 0, 2], K[:, 1, 1], K[:, 1, 2]
    dW = np.stack([fx[:, None, None] * Vm[..., 0, :], fy[:, None, None] * Vm[..., 1, :],
                   cx[:, None, None] * Vm[..., 0, :] + cy[:, None, None] * Vm[..., 1, :] +
                   Vm[..., 2, :]], -2)  # [C,N,3,3] rows, columns = (t0, t1, mc)
    vRS = np.einsum("cji,cnjk->cnik", R, dW)  # R^T dW
    sgn = np.where(-(nz * mc).sum(-1) > 0, f32(1.0), f32(-1.0))
    vtn = np.einsum("cji,cnj->cni", R, _f(v_normals)) * sgn[..., None]
    s = _f(scales)
    dR = np.stack([vRS[..., 0] * s[None, :, 0:1], vRS[..., 1] * s[None, :, 1:2], vtn], -1)
    vq = quat_to_R_vjp(np.broadcast_to(_f(quats), dR.shape[:2] + (4,)), dR)
    vs0 = (vRS[..., 0] * Rq[None, :, :, 0]).sum(-1)
    vs1 = (vRS[..., 1] * Rq[None, :, :, 1]).sum(-1)
    valid = (np.asarray(radii) > 0)[..., None]
    v_means = np.where(valid, vRS[..., 2], 0).sum(0).astype(f32)
    v_quats = np.where(valid, vq, 0).sum(0).astype(f32)
    v_scales = np.where(valid, np.stack([vs0, vs1, np.zeros_like(vs0)], -1), 0).sum(0)
    return v_means, v_quats, v_scales.astype(f32)


def _tiles(offsets, n_isects):
    flat = np.asarray(offsets, np.int64).reshape(-1)
    return flat, np.append(flat[1:], n_isects)


def _eval(m, x, y, op, px, py):
    """RasterizeToPixels2DGSFwd.cu:333-361 for one record over pixel vectors."""
    hu = [px * m[6 + i] - m[i] for i in range(3)]
    hv = [py * m[6 + i] - m[3 + i] for i in range(3)]
    rc = [hu[1] * hv[2] - hu[2] * hv[1], hu[2] * hv[0] - hu[0] * hv[2],
          hu[0] * hv[1] - hu[1] * hv[0]]
    with np.errstate(all="ignore"):
        s = (rc[0] / rc[2], rc[1] / rc[2])
        g3 = s[0] * s[0] + s[1] * s[1]
        dx, dy = x - px, y - py
        g2 = FILTER_INV_SQUARE * (dx * dx + dy * dy)
        sigma = f32(0.5) * np.minimum(g3, g2)
        vis = np.exp(-sigma).astype(f32)
        alpha = np.minimum(ALPHA_MAX, op * vis)
        ok = (rc[2] != 0) & ~(sigma < 0) & ~(alpha < ALPHA_MIN)
    return dict(hu=hu, hv=hv, rc=rc, s=s, g3=g3, g2=g2, vis=vis, alpha=alpha, ok=ok, dx=dx, dy=dy)


def raster2dgs_fwd(means2d, ray_transforms, colors, opacities, normals, backgrounds, masks, W, H,
                   ts, offsets, flatten_ids):
    """RasterizeToPixels2DGSFwd.cu:18-452.  Returns render_colors[C,H,W,D],
    alphas[C,H,W,1], normals[C,H,W,3], distort[C,H,W,1], median[C,H,W,1],
    last_ids i32[C,H,W], median_ids i32[C,H,W]."""
    C, th, tw = offsets.shape
    D = colors.shape[-1]
    m2 = _f(means2d).reshape(-1, 2)
    rt = _f(ray_transforms).reshape(-1, 9)
    cl = _f(colors).reshape(-1, D)
    op = _f(opacities).reshape(-1)
    nr = _f(normals).reshape(-1, 3)
    fids = np.asarray(flatten_ids, np.int64)
    starts, ends = _tiles(offsets, len(fids))
    oc = np.zeros((C, H, W, D), f32)
    oa = np.zeros((C, H, W, 1), f32)
    on = np.zeros((C, H, W, 3), f32)
    od = np.zeros((C, H, W, 1), f32)
    om = np.zeros((C, H, W, 1), f32)
    ol = np.zeros((C, H, W), np.int32)
    omi = np.zeros((C, H, W), np.int32)
    ly, lx = np.meshgrid(np.arange(ts), np.arange(ts), indexing="ij")
    for t in range(C * th * tw):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        pyi, pxi = (ly + ty * ts).reshape(-1), (lx + tx * ts).reshape(-1)
        inside = (pyi < H) & (pxi < W)
        if not inside.any():
            continue
        pyi, pxi = pyi[inside], pxi[inside]
        P = pyi.size
        if masks is not None and not masks[c, ty, tx]:
            oc[c, pyi, pxi] = 0 if backgrounds is None else _f(backgrounds)[c]
            continue
        px, py = pxi.astype(f32) + f32(0.5), pyi.astype(f32) + f32(0.5)
        T = np.ones(P, f32)
        done = np.zeros(P, bool)
        col = np.zeros((P, D), f32)
        nrm = np.zeros((P, 3), f32)
        dist = np.zeros(P, f32)
        avd = np.zeros(P, f32)
        med = np.zeros(P, f32)
        cur = np.zeros(P, np.int32)
        mid = np.zeros(P, np.int32)
        for j in range(starts[t], ends[t]):
            if done.all():
                break
            g = fids[j]
            h = _eval(rt[g], m2[g, 0], m2[g, 1], op[g], px, py)
            act = ~done & h["ok"]
            nT = T * (f32(1.0) - h["alpha"])
            stop = act & (nT <= T_MIN)
            done |= stop
            act &= ~stop
            vis = np.where(act, h["alpha"] * T, 0).astype(f32)
            col += vis[:, None] * cl[g][None]
            nrm += vis[:, None] * nr[g][None]
            depth = cl[g, D - 1]
            dist = np.where(act, dist + f32(2.0) * (vis * depth * (f32(1.0) - T) - vis * avd),
                            dist).astype(f32)
            avd = np.where(act, avd + vis * depth, avd).astype(f32)
            upd = act & (T > 0.5)
            med = np.where(upd, depth, med).astype(f32)
            mid = np.where(upd, j, mid).astype(np.int32)
            cur = np.where(act, j, cur).astype(np.int32)
            T = np.where(act, nT, T).astype(f32)
        if backgrounds is not None:
            col = col + T[:, None] * _f(backgrounds)[c][None]
        oc[c, pyi, pxi] = col
        oa[c, pyi, pxi, 0] = f32(1.0) - T
        on[c, pyi, pxi] = nrm
        od[c, pyi, pxi, 0] = dist
        om[c, pyi, pxi, 0] = med
        ol[c, pyi, pxi] = cur
        omi[c, pyi, pxi] = mid
    return oc, oa, on, od, om, ol, omi


def raster2dgs_bwd(means2d, ray_transforms, colors, opacities, normals, backgrounds, masks, W, H,
                   ts, offsets, flatten_ids, render_colors, render_alphas, last_ids, median_ids,
                   v_render_colors, v_render_alphas, v_render_normals, v_render_distort,
                   v_render_median, absgrad=False):
    """RasterizeToPixels2DGSBwd.cu:16-700.  Returns v_means2d, v_ray_transforms,
    v_colors, v_opacities, v_normals, v_densify, v_backgrounds (None without
    backgrounds), v_means2d_abs (None unless absgrad)."""
    C, th, tw = offsets.shape
    D = colors.shape[-1]
    m2 = _f(means2d).reshape(-1, 2)
    rt = _f(ray_transforms).reshape(-1, 9)
    cl = _f(colors).reshape(-1, D)
    op = _f(opacities).reshape(-1)
    nr = _f(normals).reshape(-1, 3)
    G = op.size
    fids = np.asarray(flatten_ids, np.int64)
    starts, ends = _tiles(offsets, len(fids))
    vm = np.zeros((G, 2), f32)
    vab = np.zeros((G, 2), f32)
    vrt = np.zeros((G, 9), f32)
    vcl = np.zeros((G, D), f32)
    vop = np.zeros(G, f32)
    vnr = np.zeros((G, 3), f32)
    rcol, ra = _f(render_colors), _f(render_alphas)
    vrc, vra, vrn = _f(v_render_colors), _f(v_render_alphas), _f(v_render_normals)
    vrd = None if v_render_distort is None else _f(v_render_distort)
    vrm = None if v_render_median is None else _f(v_render_median)
    bg = None if backgrounds is None else _f(backgrounds)
    ly, lx = np.meshgrid(np.arange(ts), np.arange(ts), indexing="ij")
    for t in range(C * th * tw):
        c, rem = divmod(t, th * tw)
        ty, tx = divmod(rem, tw)
        if masks is not None and not masks[c, ty, tx]:
            continue
        pyi, pxi = (ly + ty * ts).reshape(-1), (lx + tx * ts).reshape(-1)
        inside = (pyi < H) & (pxi < W)
        if not inside.any():
            continue
        pyi, pxi = pyi[inside], pxi[inside]
        px, py = pxi.astype(f32) + f32(0.5), pyi.astype(f32) + f32(0.5)
        Tf = f32(1.0) - ra[c, pyi, pxi, 0]
        T = Tf.copy()
        binf = last_ids[c, pyi, pxi]
        medi = median_ids[c, pyi, pxi]
        vc = vrc[c, pyi, pxi]
        va = vra[c, pyi, pxi, 0]
        vn = vrn[c, pyi, pxi]
        vd = np.zeros_like(Tf) if vrd is None else vrd[c, pyi, pxi, 0]
        vmed = np.zeros_like(Tf) if vrm is None else vrm[c, pyi, pxi, 0]
        buf = np.zeros_like(vc)
        bufn = np.zeros_like(vn)
        acc_d = rcol[c, pyi, pxi, D - 1]
        acc_w = ra[c, pyi, pxi, 0]
        accd_b, accw_b, dist_b = acc_d.copy(), acc_w.copy(), np.zeros_like(Tf)
        bg_dot = np.zeros_like(Tf) if bg is None else (vc * bg[c][None]).sum(-1, dtype=f32)
        end = min(ends[t], int(binf.max()) + 1)
        for j in range(end - 1, starts[t] - 1, -1):
            g = fids[j]
            h = _eval(rt[g], m2[g, 0], m2[g, 1], op[g], px, py)
            valid = (j <= binf) & h["ok"]
            if not valid.any():
                continue
            al = h["alpha"]
            vcol = np.zeros_like(vc)
            vcol[:, D - 1] += np.where(j == medi, vmed, 0)
            with np.errstate(all="ignore"):
                rr = f32(1.0) / (f32(1.0) - al)
            T = np.where(valid, T * rr, T).astype(f32)
            fac = al * T
            vcol += fac[:, None] * vc
            v_alpha = ((cl[g][None] * T[:, None] - buf * rr[:, None]) * vc).sum(-1, dtype=f32)
            vnrm = fac[:, None] * vn
            v_alpha += ((nr[g][None] * T[:, None] - bufn * rr[:, None]) * vn).sum(-1, dtype=f32)
            v_alpha += Tf * rr * va
            v_alpha += -Tf * rr * bg_dot
            depth = cl[g, D - 1]
            dl_dw = f32(2.0) * (f32(2.0) * (depth * accw_b - accd_b) + (acc_d - depth * acc_w))
            v_alpha += (dl_dw * T - dist_b * rr) * vd
            accd_b = np.where(valid, accd_b - fac * depth, accd_b).astype(f32)
            accw_b = np.where(valid, accw_b - fac, accw_b).astype(f32)
            dist_b = np.where(valid, dist_b + dl_dw * fac, dist_b).astype(f32)
            vcol[:, D - 1] += f32(2.0) * fac * (f32(2.0) - f32(2.0) * T - acc_w + fac) * vd
            grad_ok = valid & (op[g] * h["vis"] <= ALPHA_MAX)
            vG = op[g] * v_alpha
            use3 = grad_ok & (h["g3"] <= h["g2"])
            use2 = grad_ok & ~(h["g3"] <= h["g2"])
            s, rc, hu, hv = h["s"], h["rc"], h["hu"], h["hv"]
            with np.errstate(all="ignore"):
                vsx, vsy = vG * -h["vis"] * s[0], vG * -h["vis"] * s[1]
                ax, ay = vsx / rc[2], vsy / rc[2]
                vr = [ax, ay, -(ax * s[0] + ay * s[1])]
                vhu = [hv[1] * vr[2] - hv[2] * vr[1], hv[2] * vr[0] - hv[0] * vr[2],
                       hv[0] * vr[1] - hv[1] * vr[0]]
                vhv = [vr[1] * hu[2] - vr[2] * hu[1], vr[2] * hu[0] - vr[0] * hu[2],
                       vr[0] * hu[1] - vr[1] * hu[0]]
            vM = np.stack([-vhu[0], -vhu[1], -vhu[2], -vhv[0], -vhv[1], -vhv[2],
                           px * vhu[0] + py * vhv[0], px * vhu[1] + py * vhv[1],
                           px * vhu[2] + py * vhv[2]], -1)
            vxy = np.stack([vG * (-h["vis"] * FILTER_INV_SQUARE * h["dx"]),
                            vG * (-h["vis"] * FILTER_INV_SQUARE * h["dy"])], -1)
            vrt[g] += np.where(use3[:, None], vM, 0).sum(0, dtype=f32)
            vxy = np.where(use2[:, None], vxy, 0)
            vm[g] += vxy.sum(0, dtype=f32)
            vab[g] += np.abs(vxy).sum(0, dtype=f32)
            vop[g] += np.where(grad_ok, h["vis"] * v_alpha, 0).sum(dtype=f32)
            vcl[g] += np.where(valid[:, None], vcol, 0).sum(0, dtype=f32)
            vnr[g] += np.where(valid[:, None], vnrm, 0).sum(0, dtype=f32)
            buf = np.where(valid[:, None], buf + cl[g][None] * fac[:, None], buf).astype(f32)
            bufn = np.where(valid[:, None], bufn + nr[g][None] * fac[:, None], bufn).astype(f32)
    v_densify = np.stack([vrt[:, 2] * rt[:, 8], vrt[:, 5] * rt[:, 8]], -1).astype(f32)
    v_bg = None
    if bg is not None:
        v_bg = (vrc * (f32(1.0) - ra)).sum((1, 2), dtype=f32)
    shp = means2d.shape[:-1]
    return (vm.reshape(shp + (2,)), vrt.reshape(shp + (3, 3)), vcl.reshape(shp + (D,)),
            vop.reshape(shp), vnr.reshape(shp + (3,)), v_densify.reshape(shp + (2,)), v_bg,
            vab.reshape(shp + (2,)) if absgrad else None)
