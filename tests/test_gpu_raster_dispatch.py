"""GPU: the 16x16 rasterizer's data layout and dispatch choices change speed
only, never results.

* render records (gsplat_hip_rasterize_pack_records, ABI 15): the forward
  through the packed 64-B records is bit-identical to the forward gathering
  the four attribute arrays (the same floats reach the same arithmetic), and
  the backward agrees up to the order of its float atomics; the same for
  records and gradient rows indexed by depth rank (ABI 27);
* the forward's dispatch order (tile_order_kernel): a permutation of the
  tiles, heaviest bucket first;
* split heavy tiles (GSPLAT_HIP_FWD_SPLIT): the images of the unsplit
  forward up to chunk-product rounding, and against the oracle; the chunks'
  hand-off of transmittance products inside the one launch gives the same
  bits as every chunk computing the earlier products itself.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _scene(N=20000, W=640, H=480, seed=3):
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * torch.tensor([1.6, 1.2, 0.6])
    means[:, 2] += 4.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.08 + 0.004
    opac = torch.rand(N, generator=g)
    colors = torch.rand(N, 3, generator=g)
    vm = torch.eye(4)[None]
    K = torch.tensor([[500.0, 0, W / 2], [0, 500.0, H / 2], [0, 0, 1]])[None]
    return [x.to(DEV) for x in (means, quats, scales, opac, colors, vm, K)], W, H


def _render(ins, W, H, records, mode="RGB"):
    import gsplat_hip
    from gsplat_hip import _wrapper
    saved = _wrapper.RECORDS
    _wrapper.RECORDS = records
    try:
        leaves = [x.clone().requires_grad_(True) for x in ins[:5]]
        rc, ra, meta = gsplat_hip.rasterization(*leaves, ins[5], ins[6], W, H, packed=False,
                                                render_mode=mode)
        g = torch.Generator(device=DEV).manual_seed(1)
        w = torch.rand(rc.shape, generator=g, device=DEV)
        (rc * w).sum().backward()
        torch.cuda.synchronize()
        return rc.detach(), ra.detach(), meta, [x.grad for x in leaves]
    finally:
        _wrapper.RECORDS = saved


NAMES = ["means", "quats", "scales", "opacities", "colors"]


def _check_within_spread(g_ref, g_ref2, g_alt, what):
    """The alternative layout's gradients differ from the reference layout's
    by no more than the reference's own run-to-run noise: two runs of the same
    configuration differ because the backward's float atomics land in a
    different order each time.  Measured (profiles/r5/spread.txt): the
    per-input maxima of that noise are a few ulps of the sums and heavy-tailed
    -- layout-vs-layout over run-to-run ratios up to 5 in one run, every
    difference below 2.1e-6 of the input's largest gradient -- so the bar is
    4x the measured spread or 1e-5 of the largest value, whichever is larger
    (10x tighter than round 4's fixed 1e-4; an indexing error moves whole
    rows by O(1))."""
    for a, a2, b, name in zip(g_ref, g_ref2, g_alt, NAMES):
        scale = a.abs().max().item()
        spread = (a2 - a).abs().max().item()
        err = (b - a).abs().max().item()
        print(f"{what} {name}: err {err:.3e} spread {spread:.3e} max {scale:.3e}")
        assert err <= max(4.0 * spread, 1e-5 * scale) + 1e-12, (what, name, err, spread, scale)


@pytest.mark.parametrize("mode", ["RGB", "RGB+D"])
def test_records_match_plain_gathers(mode):
    ins, W, H = _scene()
    rc0, ra0, m0, g0 = _render(ins, W, H, False, mode)
    _, _, _, g0b = _render(ins, W, H, False, mode)
    rc1, ra1, m1, g1 = _render(ins, W, H, True, mode)
    assert m0["flatten_ids"].numel() > 50000
    assert torch.equal(rc0, rc1) and torch.equal(ra0, ra1)
    _check_within_spread(g0, g0b, g1, f"records {mode}")


def _render_ranks(ins, W, H, ranks, **kw):
    import gsplat_hip
    from gsplat_hip import _wrapper
    saved = _wrapper.RANKS
    _wrapper.RANKS = ranks
    try:
        leaves = [x.clone().requires_grad_(True) for x in ins[:5]]
        rc, ra, meta = gsplat_hip.rasterization(*leaves, ins[5], ins[6], W, H, packed=False, **kw)
        g = torch.Generator(device=DEV).manual_seed(1)
        w = torch.rand(rc.shape, generator=g, device=DEV)
        (rc * w).sum().backward()
        torch.cuda.synchronize()
        return rc.detach(), ra.detach(), meta, [x.grad for x in leaves]
    finally:
        _wrapper.RANKS = saved


@pytest.mark.parametrize("capped", [False, True])
def test_rank_indexed_rows_match_gaussian_rows(capped):
    """Render records and gradient rows indexed by the visible Gaussians'
    depth rank (GSPLAT_HIP_RANKS, ABI 27): the same records reach the same
    arithmetic, so the forward is bit-identical and the backward agrees up to
    its float atomics' order -- within twice the spread of two runs of the
    Gaussian-indexed layout; meta["flatten_ids"] keeps the Gaussian ids."""
    ins, W, H = _scene()
    kw = {}
    if capped:
        kw = dict(_isect_capacity=400000,
                  _isect_status=torch.zeros(1, dtype=torch.int32, device=DEV))
    rc0, ra0, m0, g0 = _render_ranks(ins, W, H, False, **kw)
    _, _, _, g0b = _render_ranks(ins, W, H, False, **kw)
    rc1, ra1, m1, g1 = _render_ranks(ins, W, H, True, **kw)
    # (capacity-sized arrays: the first counts[0] entries are the isects)
    n = int(m0["isect_counts"][0]) if capped else m0["flatten_ids"].numel()
    assert torch.equal(m0["flatten_ids"][:n], m1["flatten_ids"][:n])
    assert torch.equal(m0["isect_ids"][:n], m1["isect_ids"][:n])
    assert torch.equal(rc0, rc1) and torch.equal(ra0, ra1)
    _check_within_spread(g0, g0b, g1, f"ranks capped={capped}")
    assert n > 50000


def test_dispatch_order_is_heaviest_first_permutation():
    """gsplat_hip_rasterize_prepare's tile order (tile_order_kernel): a
    permutation of the tiles, buckets of >= 2048 / >= 1024 / >= 512 isects and
    the rest in that order, lane order inside a bucket."""
    from gsplat_hip import _lib
    from gsplat_hip._wrapper import _ptr, _stream
    import gsplat_hip
    ins, W, H = _scene(N=60000, W=1280, H=720)
    with torch.no_grad():
        _, _, meta = gsplat_hip.rasterization(*ins[:5], ins[5], ins[6], W, H, packed=False)
    offs = meta["isect_offsets"].contiguous()
    n = meta["flatten_ids"].numel()
    C, th, tw = offs.shape
    nt = C * th * tw
    D = 3
    old = _lib.query("gsplat_hip_debug_set_fwd_split", 0)  # no split area after the order
    old_flags = _lib.query("gsplat_hip_debug_set_flags", 16)  # the per-tile order
    try:
        sb = int(_lib.query("gsplat_hip_rasterize_fwd_state_bytes", C, D, 16, tw, th, n))
        state = torch.full((sb // 4,), -7, dtype=torch.int32, device=DEV)
        _lib.call("gsplat_hip_rasterize_prepare", C, D, 16, tw, th, _ptr(offs), n, None,
                  _ptr(state), sb, _stream())
        torch.cuda.synchronize()
    finally:
        _lib.query("gsplat_hip_debug_set_fwd_split", old)
        _lib.query("gsplat_hip_debug_set_flags", old_flags)
    # the order area (256-B aligned, room for the XCD-grouped order's slots:
    # 2 nt + 64 entries) is the last part of the state
    order_ints = (4 * (2 * nt + 64) + 255) // 256 * 64
    order = state[-order_ints:][:nt].cpu().numpy()
    assert np.array_equal(np.sort(order), np.arange(nt)), "not a permutation"
    o = offs.flatten().cpu().numpy().astype(np.int64)
    cnt = np.diff(np.concatenate([o, [n]]))
    assert (cnt[order] >= 512).any(), "scene has no heavy tiles"
    b = np.where(cnt[order] >= 2048, 0, np.where(cnt[order] >= 1024, 1,
                                                  np.where(cnt[order] >= 512, 2, 3)))
    assert np.all(np.diff(b) >= 0), "buckets not heaviest first"
    for bk in range(4):  # lane t % 1024 holds tiles t, t + 1024, ...: lane-major
        t = order[b == bk].astype(np.int64)
        assert np.all(np.diff((t % 1024) * 16 + t // 1024) > 0), f"bucket {bk}: not lane order"


def _heavy_scene(N=60000, W=320, H=240, seed=5):
    """Many large Gaussians over a small image: tiles with thousands of isects."""
    g = torch.Generator().manual_seed(seed)
    means = torch.randn(N, 3, generator=g) * torch.tensor([1.0, 0.8, 0.5])
    means[:, 2] += 5.0
    quats = torch.randn(N, 4, generator=g)
    scales = torch.rand(N, 3, generator=g) * 0.12 + 0.01
    opac = torch.rand(N, generator=g) * 0.3  # low opacity: long tiles before saturation
    colors = torch.rand(N, 3, generator=g)
    vm = torch.eye(4)[None]
    K = torch.tensor([[300.0, 0, W / 2], [0, 300.0, H / 2], [0, 0, 1]])[None]
    return [x.to(DEV) for x in (means, quats, scales, opac, colors, vm, K)], W, H


def _render_split(ins, W, H, split, mode="RGB"):
    from gsplat_hip import _lib
    old = _lib.query("gsplat_hip_debug_set_fwd_split", split)
    try:
        return _render(ins, W, H, True, mode)
    finally:
        _lib.query("gsplat_hip_debug_set_fwd_split", old)


@pytest.mark.parametrize("split,mode", [(2048, "RGB"), (300, "RGB+D"), (64, "RGB")])
def test_split_forward_matches_unsplit(split, mode):
    """Tiles above `split` isects rendered as parallel chunks (transmittance
    products, chunk compositing, combine) give the unsplit forward's images up
    to the float rounding of the chunk products (and the threshold flips it can
    cause), and the backward -- which reads the chunk state the split forward
    writes -- the same gradients."""
    ins, W, H = _heavy_scene()
    rc0, ra0, m0, g0 = _render_split(ins, W, H, 0, mode)
    rc1, ra1, m1, g1 = _render_split(ins, W, H, split, mode)
    offs = m0["isect_offsets"].flatten().long()
    n = m0["flatten_ids"].numel()
    cnt = torch.diff(torch.cat([offs, torch.tensor([n], device=DEV)]))
    assert int((cnt > split).sum()) >= 4, "scene has too few heavy tiles"
    from test_gpu_parity import close_most
    close_most(rc1, rc0, 1e-5, 1e-5, "colors", max_frac=1e-3)
    close_most(ra1, ra0, 1e-5, 1e-5, "alphas", max_frac=1e-3)
    for a, b, name in zip(g1, g0, ["means", "quats", "scales", "opacities", "colors"]):
        scale = max(1e-12, float(b.abs().max()))
        close_most(a, b, 1e-3, 1e-4 * scale, name, max_frac=2e-3, rows=True,
                   out_bound=0.05 * scale)


def test_split_handoff_equals_local_products():
    """A chunk of a split tile takes the earlier chunks' transmittance
    products from their workgroups (sc1 hand-off, bounded wait) or, when one
    is late, computes it itself: both give the same bits (debug flag bit 1
    forces the local path for every chunk)."""
    from gsplat_hip import _lib
    ins, W, H = _heavy_scene()
    rc0, ra0, m0, g0 = _render_split(ins, W, H, 300)
    old = _lib.query("gsplat_hip_debug_set_flags", 2)
    try:
        rc1, ra1, m1, g1 = _render_split(ins, W, H, 300)
    finally:
        _lib.query("gsplat_hip_debug_set_flags", old)
    offs = m0["isect_offsets"].flatten().long()
    n = m0["flatten_ids"].numel()
    cnt = torch.diff(torch.cat([offs, torch.tensor([n], device=DEV)]))
    assert int((cnt > 2048).sum()) >= 4, "scene has too few multi-chunk tiles"
    assert torch.equal(rc0, rc1) and torch.equal(ra0, ra1)
    for a, b, name in zip(g1, g0, ["means", "quats", "scales", "opacities", "colors"]):
        scale = max(1e-12, float(b.abs().max()))
        assert float((a - b).abs().max()) <= 1e-5 * scale, name


def test_split_forward_vs_oracle():
    """The split forward against the CPU oracle on a scene with heavy tiles."""
    import numpy as np
    from oracle import gsplat_oracle as O
    from gsplat_hip import _lib
    import gsplat_hip
    default = _lib.query("gsplat_hip_debug_set_fwd_split", 200)
    try:
        ins, W, H = _heavy_scene(N=20000, W=128, H=96, seed=7)
        with torch.no_grad():
            rc, ra, meta = gsplat_hip.rasterization(*ins[:5], ins[5], ins[6], W, H, packed=False)
    finally:
        _lib.query("gsplat_hip_debug_set_fwd_split", default)
    offs = meta["isect_offsets"].cpu().numpy()
    fids = meta["flatten_ids"].cpu().numpy()
    n = fids.size
    cnt = np.diff(np.concatenate([offs.ravel(), [n]]))
    assert (cnt > 200).sum() >= 4
    m2 = meta["means2d"].cpu().numpy()
    cn = meta["conics"].cpu().numpy()
    op = meta["opacities"].cpu().numpy()
    cols = ins[4].cpu().numpy()[None]
    oc, oa, _ = O.raster_fwd(m2, cn, cols, op, None, W, H, 16, offs, fids)
    from test_gpu_parity import close_most
    close_most(ra, oa, 1e-4, 1e-4, "alphas", max_frac=1e-3)
    close_most(rc, oc, 1e-4, 1e-4, "colors", max_frac=1e-3)


@pytest.mark.parametrize("W,H", [(640, 480), (200, 150), (1000, 24)])
def test_xcd_grouped_order_changes_nothing(W, H):
    """The XCD-grouped dispatch order (tile_order_grouped_kernel, the default;
    debug flag bit 4 restores the per-tile order): 2x2 groups of tiles,
    heaviest group first, a group's tiles in slots of one XCD, empty slots at
    the image edges (odd tile counts) -- the forward's images bit for bit, the
    backward at the run-to-run spread of the float atomics.  The same flag
    selects the backward's work-item order (runs of four items per XCD by
    default, the list order with bit 4), which the gradients cover."""
    from gsplat_hip import _lib
    ins, _, _ = _scene(W=W, H=H)
    old_split = _lib.query("gsplat_hip_debug_set_fwd_split", 0)  # the unsplit forward
    try:
        rc0, ra0, _, g0 = _render(ins, W, H, True)
        rc0b, _, _, g0b = _render(ins, W, H, True)
        old = _lib.query("gsplat_hip_debug_set_flags", 16)
        try:
            rc1, ra1, _, g1 = _render(ins, W, H, True)
        finally:
            _lib.query("gsplat_hip_debug_set_flags", old)
    finally:
        _lib.query("gsplat_hip_debug_set_fwd_split", old_split)
    assert torch.equal(rc0, rc1) and torch.equal(ra0, ra1) and torch.equal(rc0, rc0b)
    _check_within_spread(g0, g0b, g1, f"grouped order {W}x{H}")
