"""Generate golden input/output vectors from the REFERENCE Triton kernels.

Run in the build container only (needs /root/reference and triton):

    python tests/golden/make_golden.py

The reference's own Triton backend (`gsplat/triton_impl/*`) is executed on the
CPU with `TRITON_INTERPRET=1`.  Four harness-side shims are applied (SURVEY.md
§8c); nothing under /root/reference is modified or copied:

1. `jaxtyping` (annotation-only import, e.g. fused_projection_fwd.py:7) is
   stubbed.
2. Python `bool` kernel arguments are mapped to `np.bool_` for the interpreter
   (fused_projection_fwd.py:31, rasterize_to_pixels_bwd.py:55).
3. `libdevice.{rsqrt,fast_expf,fast_logf}` return None under the interpreter;
   they are rebound to `tl.rsqrt/tl.exp/tl.log`.
4. `gsplat.triton_impl.radix_sort` (nvcc JIT of CUB, radix_sort/__init__.py:10)
   is replaced by a *stable* torch sort restricted to the low `n_bits` key bits
   -- the published semantics of cub::DeviceRadixSort::SortPairs.

Only the produced arrays (inputs + outputs) are committed, as .npz files next
to this script.  The GPU box never runs this file.
"""

import math
import os
import sys
import time
import types

os.environ["TRITON_INTERPRET"] = "1"

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ---------------------------------------------------------------- shims ----
def _install_shims():
    # (1) jaxtyping stub
    jt = types.ModuleType("jaxtyping")

    class _Ann:
        def __getitem__(self, item):
            return object

    for n in ("Float", "Int32", "Int64", "Int", "Bool", "Float32"):
        setattr(jt, n, _Ann())
    sys.modules["jaxtyping"] = jt

    import triton.language as tl
    import triton.runtime.interpreter as interp
    from triton.language.extra import libdevice

    # (2) bool args
    _orig = interp._implicit_cvt

    def _cvt(arg):
        if isinstance(arg, bool):
            arg = np.bool_(arg)
        return _orig(arg)

    interp._implicit_cvt = _cvt

    # (3) libdevice fast-math entry points
    libdevice.rsqrt = lambda x, **kw: tl.rsqrt(x)
    libdevice.fast_expf = lambda x, **kw: tl.exp(x)
    libdevice.fast_logf = lambda x, **kw: tl.log(x)

    # package root without executing gsplat/__init__.py (it pulls in
    # compression/strategy extras that are not needed here)
    pkg = types.ModuleType("gsplat")
    pkg.__path__ = [os.path.join(REF, "gsplat")]
    sys.modules["gsplat"] = pkg

    # (4) radix sort stand-in: stable sort on the low n_bits bits
    rs = types.ModuleType("gsplat.triton_impl.radix_sort")

    def radix_sort(keys, values, n_bits):
        mask = (1 << n_bits) - 1 if n_bits < 63 else -1
        k = keys & mask
        order = torch.sort(k, stable=True).indices
        return keys[order], values[order]

    rs.radix_sort = radix_sort
    sys.modules["gsplat.triton_impl.radix_sort"] = rs


_install_shims()
sys.path.insert(0, REF)

from gsplat.triton_impl import _wrapper as W  # noqa: E402
from gsplat.triton_impl._wrapper import load_triton_kernel  # noqa: E402
from gsplat._helper import load_test_data  # noqa: E402


def save(name, **arrs):
    out = {}
    for k, v in arrs.items():
        if v is None:
            continue
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu().numpy()
        out[k] = np.asarray(v)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"  wrote {name}.npz ({os.path.getsize(path)/1024:.1f} KiB)")


def garden(n_keep, seed, downscale=1, scale_mul=1.0):
    """load_test_data() semantics (gsplat/_helper.py:9-55) on CPU, subsampled."""
    torch.manual_seed(seed)
    means, quats, scales, opac, colors, viewmats, Ks, W_, H_ = load_test_data(
        data_path=os.path.join(REF, "assets/test_garden.npz"), device="cpu"
    )
    g = torch.Generator().manual_seed(seed + 1)
    sel = torch.randperm(len(means), generator=g)[:n_keep].sort().values
    means, quats, scales, opac, colors = (
        means[sel], quats[sel], scales[sel] * scale_mul, opac[sel], colors[sel]
    )
    Ks = Ks.clone()
    if downscale != 1:
        Ks[:, :2, :] /= downscale
        W_, H_ = int(math.ceil(W_ / downscale)), int(math.ceil(H_ / downscale))
    return means, quats, scales, opac, colors, viewmats, Ks, W_, H_


def synthetic_m1(seed=0, N=1000, C=1, W_=256, H_=256):
    """SURVEY.md §8d config M1."""
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * 0.8
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.05 + 0.005
    opac = torch.rand(N, generator=g)
    sh = torch.randn(N, 16, 3, generator=g) * 0.3
    viewmats = torch.eye(4)[None].repeat(C, 1, 1)
    Ks = torch.tensor([[200.0, 0, W_ / 2], [0, 200.0, H_ / 2], [0, 0, 1]])[None].repeat(C, 1, 1)
    if C > 1:
        for c in range(1, C):
            viewmats[c, :3, 3] = torch.randn(3, generator=g) * 0.2
    return means, quats, scales, opac, sh, viewmats, Ks, W_, H_


# --------------------------------------------------------- projection -----
def gen_projection():
    print("projection")
    cases = []
    # garden cameras, full res, mix of in/out of frustum points
    m, q, s, o, col, vm, K, W_, H_ = garden(600, seed=42)
    cases.append(("proj_garden", m, q, s, vm, K, W_, H_, 0.01, 1e10, 0.0))
    # synthetic: points behind / near / far and off-screen (clamp branch), radius clip
    g = torch.Generator().manual_seed(7)
    N = 500
    m2 = torch.randn(N, 3, generator=g) * 2.0
    m2[:, 2] += 2.0
    q2 = torch.randn(N, 4, generator=g)
    s2 = torch.rand(N, 3, generator=g) * 0.3 + 0.01
    vm2 = torch.eye(4)[None].repeat(2, 1, 1)
    vm2[1, :3, 3] = torch.tensor([0.3, -0.2, 0.5])
    th = 0.3
    vm2[1, :3, :3] = torch.tensor([[math.cos(th), 0, math.sin(th)], [0, 1, 0], [-math.sin(th), 0, math.cos(th)]])
    K2 = torch.tensor([[150.0, 0, 100], [0, 160.0, 70], [0, 0, 1]])[None].repeat(2, 1, 1)
    cases.append(("proj_synth", m2, q2, s2, vm2, K2, 200, 140, 0.5, 6.0, 1.5))

    for name, m, q, s, vm, K, W_, H_, near, far, rclip in cases:
        for comp in (False, True):
            t0 = time.time()
            mm, qq, ss, vv = (x.clone().requires_grad_(True) for x in (m, q, s, vm))
            radii, means2d, depths, conics, comps = W.fully_fused_projection(
                mm, None, qq, ss, vv, K, W_, H_, eps2d=0.3, near_plane=near,
                far_plane=far, radius_clip=rclip, calc_compensations=comp,
            )
            g2 = torch.Generator().manual_seed(11)
            v_m2 = torch.randn(means2d.shape, generator=g2)
            v_d = torch.randn(depths.shape, generator=g2)
            v_c = torch.randn(conics.shape, generator=g2)
            v_cp = torch.randn(depths.shape, generator=g2) if comp else None
            valid = (radii > 0)
            # only valid entries carry gradient (reference bwd masks by radii>0,
            # fused_projection_bwd.py:68-69); zero the rest so the loss is finite
            loss = (torch.where(valid[..., None], means2d, 0) * v_m2).sum() \
                + (torch.where(valid, depths, 0) * v_d).sum() \
                + (torch.where(valid[..., None], conics, 0) * v_c).sum()
            if comp:
                loss = loss + (torch.where(valid, comps, 0) * v_cp).sum()
            gm, gq, gs, gv = torch.autograd.grad(loss, (mm, qq, ss, vv))
            save(f"{name}{'_comp' if comp else ''}",
                 means=m, quats=q, scales=s, viewmats=vm, Ks=K,
                 width=W_, height=H_, near=near, far=far, radius_clip=rclip, eps2d=0.3,
                 radii=radii, means2d=means2d, depths=depths, conics=conics, comps=comps,
                 v_means2d=v_m2 * valid[..., None], v_depths=v_d * valid,
                 v_conics=v_c * valid[..., None],
                 v_comps=None if v_cp is None else v_cp * valid,
                 v_means=gm, v_quats=gq, v_scales=gs, v_viewmats=gv)
            print(f"   {name} comp={comp} {time.time()-t0:.1f}s valid={int(valid.sum())}")


# ------------------------------------------------------------------ SH -----
def gen_sh():
    print("spherical harmonics")
    g = torch.Generator().manual_seed(43)
    shape = (37, 23)
    coeffs = torch.randn(*shape, 25, 3, generator=g)
    dirs = torch.randn(*shape, 3, generator=g)
    masks = torch.rand(*shape, generator=g) > 0.2
    v_colors = torch.randn(*shape, 3, generator=g)
    for d in range(5):
        t0 = time.time()
        K = max((d + 1) ** 2, 1)
        cf = coeffs[..., : (16 if d <= 3 else 25), :].clone().requires_grad_(True)
        dr = dirs.clone().requires_grad_(True)
        colors = W.spherical_harmonics(d, dr, cf, masks=masks)
        gc, gd = torch.autograd.grad((colors * v_colors).sum(), (cf, dr), allow_unused=True)
        save(f"sh_deg{d}", degree=d, coeffs=cf.detach(), dirs=dirs, masks=masks,
             colors=colors, v_colors=v_colors, v_coeffs=gc, v_dirs=gd)
        print(f"   deg {d} K={cf.shape[-2]} {time.time()-t0:.1f}s")


# --------------------------------------------------------------- isect -----
def gen_isect():
    print("isect")
    from gsplat.cuda._torch_impl import _isect_tiles, _isect_offset_encode
    cases = []
    m, q, s, o, col, vm, K, W_, H_ = garden(700, seed=50, scale_mul=0.1)
    cases.append(("isect_garden_t16", m, q, s, vm, K, W_, H_, 16))
    cases.append(("isect_garden_t4", m, q, s, vm, K, W_, H_, 4))
    # 256x256 / 16 -> 256 tiles (power of two) with C=2: the L1 landmine
    mm, qq, ss, oo, sh, vv, KK, w2, h2 = synthetic_m1(seed=3, N=400, C=2)
    cases.append(("isect_pow2_c2", mm, qq, ss, vv, KK, w2, h2, 16))
    for name, m, q, s, vm, K, W_, H_, ts in cases:
        t0 = time.time()
        radii, means2d, depths, conics, _ = W.fully_fused_projection(m, None, q, s, vm, K, W_, H_)
        tw, th = math.ceil(W_ / ts), math.ceil(H_ / ts)
        tpg, iids, fids = W.isect_tiles(means2d, radii, depths, ts, tw, th)
        offs = W.isect_offset_encode(iids, vm.shape[0], tw, th)
        # torch_impl cross-check (its tile bit width differs: L1)
        _tpg, _iids, _fids = _isect_tiles(means2d, radii, depths, ts, tw, th)
        assert torch.equal(tpg, _tpg) and torch.equal(fids, _fids), name
        # keep only valid entries for means2d (L4)
        means2d = torch.where((radii > 0)[..., None], means2d, 0.0)
        save(name, means2d=means2d, radii=radii, depths=depths, tile_size=ts,
             tile_width=tw, tile_height=th, C=vm.shape[0],
             tiles_per_gauss=tpg, isect_ids=iids, flatten_ids=fids, isect_offsets=offs)
        print(f"   {name} n_isects={len(iids)} {time.time()-t0:.1f}s")


# ------------------------------------------------------------- raster ------
def gen_raster():
    print("rasterize")
    cases = []
    m, q, s, o, col, vm, K, W_, H_ = garden(1500, seed=50, downscale=4, scale_mul=0.4)
    cases.append(("raster_garden_d3_bg", m, q, s, o, col, vm[:2], K[:2], W_, H_, 3, True))
    cases.append(("raster_garden_d4", m, q, s, o, col, vm[:1], K[:1], W_, H_, 4, False))
    cases.append(("raster_garden_d8_bg", m, q, s, o, col, vm[2:3], K[2:3], W_, H_, 8, True))
    for name, m, q, s, o, col, vm, K, W_, H_, D, use_bg in cases:
        t0 = time.time()
        C = vm.shape[0]
        radii, means2d, depths, conics, _ = W.fully_fused_projection(m, None, q, s, vm, K, W_, H_)
        ts = 16
        tw, th = math.ceil(W_ / ts), math.ceil(H_ / ts)
        tpg, iids, fids = W.isect_tiles(means2d, radii, depths, ts, tw, th)
        offs = W.isect_offset_encode(iids, C, tw, th)
        g = torch.Generator().manual_seed(99)
        colors = torch.rand(C, m.shape[0], D, generator=g)
        colors[:, :, :3] = col[None]
        opac = o[None].repeat(C, 1)
        bg = torch.rand(C, D, generator=g) if use_bg else None
        means2d = torch.where((radii > 0)[..., None], means2d, 0.0)
        conics = torch.where((radii > 0)[..., None], conics, 0.0)
        m2d, cn, cl, op = (x.clone().requires_grad_(True) for x in (means2d, conics, colors, opac))
        bgr = bg.clone().requires_grad_(True) if use_bg else None
        rc, ra = W.rasterize_to_pixels(m2d, cn, cl, op, W_, H_, ts, offs, fids,
                                       backgrounds=bgr, absgrad=True)
        # last_ids straight from the reference forward kernel launcher
        Dp = 1 << (D - 1).bit_length()
        pad = lambda x: torch.cat([x, torch.zeros(*x.shape[:-1], Dp - D)], -1) if Dp != D else x
        _, _, last_ids = load_triton_kernel("rasterize_to_pixels_fwd")(
            means2d, conics, pad(colors), opac, None if bg is None else pad(bg), None,
            W_, H_, ts, offs, fids, 8)
        v_rc = torch.randn(rc.shape, generator=g)
        v_ra = torch.randn(ra.shape, generator=g)
        ins = (m2d, cn, cl, op) + ((bgr,) if use_bg else ())
        grads = torch.autograd.grad((rc * v_rc).sum() + (ra * v_ra).sum(), ins)
        save(name, means2d=means2d, conics=conics, colors=colors, opacities=opac,
             backgrounds=bg, width=W_, height=H_, tile_size=ts, isect_offsets=offs,
             flatten_ids=fids, render_colors=rc, render_alphas=ra, last_ids=last_ids,
             v_render_colors=v_rc, v_render_alphas=v_ra,
             v_means2d=grads[0], v_conics=grads[1], v_colors=grads[2], v_opacities=grads[3],
             v_backgrounds=grads[4] if use_bg else None, v_means2d_abs=m2d.absgrad)
        print(f"   {name} {W_}x{H_} C={C} D={D} n_isects={len(fids)} {time.time()-t0:.1f}s")


# ------------------------------------------------------ end-to-end M1 ------
def gen_e2e():
    print("end-to-end rasterization() M1")
    from gsplat.rendering import rasterization
    for name, mode, C in (("e2e_m1_rgb", "RGB", 1), ("e2e_m1c2_rgbed", "RGB+ED", 2)):
        t0 = time.time()
        means, quats, scales, opac, sh, vm, K, W_, H_ = synthetic_m1(seed=0, C=C)
        ins = [x.clone().requires_grad_(True) for x in (means, quats, scales, opac, sh)]
        bg = torch.full((C, 3), 0.25)
        rc, ra, meta = rasterization(ins[0], ins[1], ins[2], ins[3], ins[4], vm, K, W_, H_,
                                     sh_degree=3, packed=False, render_mode=mode,
                                     backgrounds=bg)
        g = torch.Generator().manual_seed(5)
        v_rc = torch.randn(rc.shape, generator=g)
        v_ra = torch.randn(ra.shape, generator=g)
        meta["means2d"].retain_grad()
        grads = torch.autograd.grad((rc * v_rc).sum() + (ra * v_ra).sum(), ins)
        save(name, means=means, quats=quats, scales=scales, opacities=opac, sh=sh,
             viewmats=vm, Ks=K, width=W_, height=H_, backgrounds=bg, render_mode=mode,
             render_colors=rc, render_alphas=ra, radii=meta["radii"],
             tiles_per_gauss=meta["tiles_per_gauss"], isect_ids=meta["isect_ids"],
             flatten_ids=meta["flatten_ids"], isect_offsets=meta["isect_offsets"],
             v_render_colors=v_rc, v_render_alphas=v_ra,
             v_means=grads[0], v_quats=grads[1], v_scales=grads[2],
             v_opacities=grads[3], v_sh=grads[4])
        print(f"   {name} n_isects={len(meta['flatten_ids'])} {time.time()-t0:.1f}s")


def gen_e2e_aa():
    """rasterization() with rasterize_mode="antialiased" (the compensation
    multiply, gsplat/rendering.py:328,347-351), which the two M1 fixtures
    above leave out."""
    print("end-to-end rasterization() options")
    from gsplat.rendering import rasterization
    # antialiased, SH degree 3, RGB
    t0 = time.time()
    means, quats, scales, opac, sh, vm, K, W_, H_ = synthetic_m1(seed=3)
    ins = [x.clone().requires_grad_(True) for x in (means, quats, scales, opac, sh)]
    rc, ra, meta = rasterization(ins[0], ins[1], ins[2], ins[3], ins[4], vm, K, W_, H_,
                                 sh_degree=3, packed=False, rasterize_mode="antialiased")
    g = torch.Generator().manual_seed(6)
    v_rc = torch.randn(rc.shape, generator=g)
    v_ra = torch.randn(ra.shape, generator=g)
    grads = torch.autograd.grad((rc * v_rc).sum() + (ra * v_ra).sum(), ins)
    save("e2e_m1_aa", means=means, quats=quats, scales=scales, opacities=opac, sh=sh,
         viewmats=vm, Ks=K, width=W_, height=H_, render_colors=rc, render_alphas=ra,
         radii=meta["radii"], isect_ids=meta["isect_ids"], flatten_ids=meta["flatten_ids"],
         opacities_eff=meta["opacities"], v_render_colors=v_rc, v_render_alphas=v_ra,
         v_means=grads[0], v_quats=grads[1], v_scales=grads[2], v_opacities=grads[3],
         v_sh=grads[4])
    print(f"   e2e_m1_aa n_isects={len(meta['flatten_ids'])} {time.time()-t0:.1f}s")


def gen_e2e_d40():
    """40 colour channels (no SH): two chunks, 32 + 8, with backgrounds
    (gsplat/rendering.py:544-572); a 96x96 image keeps the fixture small."""
    from gsplat.rendering import rasterization
    t0 = time.time()
    means, quats, scales, opac, _, vm, K, W_, H_ = synthetic_m1(seed=4, N=600, W_=96, H_=96)
    D = 40
    cols = torch.rand(len(means), D, generator=torch.Generator().manual_seed(7))
    bg = torch.linspace(0.0, 1.0, D)[None]
    ins = [x.clone().requires_grad_(True) for x in (means, quats, scales, opac, cols)]
    rc, ra, meta = rasterization(ins[0], ins[1], ins[2], ins[3], ins[4], vm, K, W_, H_,
                                 packed=False, backgrounds=bg, channel_chunk=32)
    g = torch.Generator().manual_seed(8)
    v_rc = torch.randn(rc.shape, generator=g)
    v_ra = torch.randn(ra.shape, generator=g)
    grads = torch.autograd.grad((rc * v_rc).sum() + (ra * v_ra).sum(), ins)
    save("e2e_m1_d40", means=means, quats=quats, scales=scales, opacities=opac, colors=cols,
         viewmats=vm, Ks=K, width=W_, height=H_, backgrounds=bg, render_colors=rc,
         render_alphas=ra, radii=meta["radii"], isect_ids=meta["isect_ids"],
         flatten_ids=meta["flatten_ids"], v_render_colors=v_rc, v_render_alphas=v_ra,
         v_means=grads[0], v_quats=grads[1], v_scales=grads[2], v_opacities=grads[3],
         v_colors=grads[4])
    print(f"   e2e_m1_d40 n_isects={len(meta['flatten_ids'])} {time.time()-t0:.1f}s")


def gen_scene():
    """Benchmark scene: assets/test_garden.npz cropped to [-2,2]^3 exactly as
    load_test_data() does (gsplat/_helper.py:30-36) -- SfM points, colours and
    the 3 cameras.  bench.py tiles it 3x3 (scene_grid=3) into M2."""
    print("scene")
    d = np.load(os.path.join(REF, "assets/test_garden.npz"))
    means = d["means3d"].astype(np.float32)
    sel = np.all((means >= -2) & (means <= 2), axis=-1)
    np.savez_compressed(os.path.join(OUT, "garden_scene.npz"), means3d=means[sel],
                        colors=d["colors"][sel], viewmats=d["viewmats"].astype(np.float32),
                        Ks=d["Ks"].astype(np.float32), width=d["width"], height=d["height"])
    print(f"  wrote garden_scene.npz ({int(sel.sum())} points)")


if __name__ == "__main__":
    which = sys.argv[1:] or ["projection", "sh", "isect", "raster", "e2e", "scene"]
    torch.set_num_threads(8)
    for w in which:
        {"projection": gen_projection, "sh": gen_sh, "isect": gen_isect,
         "raster": gen_raster, "e2e": gen_e2e, "e2e_aa": gen_e2e_aa, "e2e_d40": gen_e2e_d40,
         "scene": gen_scene}[w]()
