"""CPU oracle for DefaultStrategy's refine step -- TEST INFRASTRUCTURE ONLY.

A numpy restatement of the reference's
  DefaultStrategy._grow_gs   gsplat/strategy/default.py:264-311
  DefaultStrategy._prune_gs  gsplat/strategy/default.py:313-340
  duplicate / split / remove gsplat/strategy/ops.py:86-211
  reset_opa                  gsplat/strategy/ops.py:214-243
including what they do to the Adam state (new rows start with zero moments,
removed rows drop theirs, reset_opa zeroes the opacity moments).  Pinned to
goldens produced by the reference's own code (`tests/golden/
make_golden_strategy.py`, `tests/test_strategy_oracle.py`).  Only `tests/`
import it.

`params` / `moments`: dicts name -> array [N, ...]; moments[name] is a pair
(exp_avg, exp_avg_sq).  `z`: the split noise [2, n_split, 3] (the reference
draws torch.randn(2, n_split, 3) inside split(), ops.py:147-152).
"""

import numpy as np

f32 = np.float32

DEFAULTS = dict(prune_opa=0.005, grow_grad2d=0.0002, grow_scale3d=0.01, prune_scale3d=0.1,
                grow_scale2d=0.05, prune_scale2d=0.15, reset_every=3000, revised_opacity=False)


def _sigmoid(x):
    return (f32(1.0) / (f32(1.0) + np.exp(-x.astype(f32)))).astype(f32)


def _rotmat(q):
    """normalized_quat_to_rotmat(F.normalize(q)) (gsplat/utils.py)."""
    q = q / np.maximum(np.linalg.norm(q, axis=-1, keepdims=True), 1e-12)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)
    return R.reshape(-1, 3, 3).astype(f32)


def _cat(*xs):
    return np.concatenate(xs, 0)


def refine(params, moments, grad2d, count, step, z, scene_scale=1.0, radii2d=None, **cfg):
    """One refine step (grow, then prune).  Returns (params, moments,
    (n_dupli, n_split, n_prune)).  radii2d: state["radii"] when the caller is
    before refine_scale2d_stop_iter (screen-size split and prune,
    default.py:283-284, 325-326), carried through duplicate / split as the
    reference's running state (ops.py:108-111, 172-176)."""
    c = dict(DEFAULTS, **cfg)
    p = {k: np.asarray(v, f32).copy() for k, v in params.items()}
    m = {k: (np.asarray(a, f32).copy(), np.asarray(b, f32).copy()) for k, (a, b) in moments.items()}
    N = len(p["means"])
    # _grow_gs (default.py:271-311)
    grads = grad2d / np.maximum(count, 1.0)
    high = grads > c["grow_grad2d"]
    small = np.exp(p["scales"]).max(-1) <= c["grow_scale3d"] * scene_scale
    dup = high & small
    split = high & ~small
    rad = None if radii2d is None else np.asarray(radii2d, f32).copy()
    if rad is not None:
        split = split | (rad > c["grow_scale2d"])
    n_dupli, n_split = int(dup.sum()), int(split.sum())
    # duplicate (ops.py:86-112): append copies, zero moments
    sel = np.nonzero(dup)[0]
    for k in p:
        p[k] = _cat(p[k], p[k][sel])
        m[k] = tuple(_cat(v, np.zeros((len(sel),) + v.shape[1:], f32)) for v in m[k])
    split = _cat(split, np.zeros(n_dupli, bool))
    if rad is not None:
        rad = _cat(rad, rad[sel])
    # split (ops.py:115-176): keep the rest, append the two children batches
    sel = np.nonzero(split)[0]
    rest = np.nonzero(~split)[0]
    assert z.shape == (2, len(sel), 3), (z.shape, len(sel))
    scales = np.exp(p["scales"][sel]).astype(f32)
    R = _rotmat(p["quats"][sel])
    samples = np.einsum("nij,nj,bnj->bni", R, scales, z.astype(f32)).astype(f32)
    for k in p:
        v = p[k]
        if k == "means":
            child = (v[sel][None] + samples).reshape(-1, 3)
        elif k == "scales":
            child = np.tile(np.log(scales * f32(1.0 / 1.6)).astype(f32), (2, 1))
        elif k == "opacities" and c["revised_opacity"]:
            o = f32(1.0) - np.sqrt(f32(1.0) - _sigmoid(v[sel]))
            child = np.tile(np.log(o / (f32(1.0) - o)).astype(f32), 2)
        else:
            child = np.concatenate([v[sel], v[sel]], 0)
        p[k] = _cat(v[rest], child.astype(f32))
        m[k] = tuple(_cat(a[rest], np.zeros((2 * len(sel),) + a.shape[1:], f32)) for a in m[k])
    if rad is not None:
        rad = _cat(rad[rest], rad[sel], rad[sel])
    # _prune_gs (default.py:313-340) + remove (ops.py:179-211)
    prune = _sigmoid(p["opacities"].reshape(-1)) < c["prune_opa"]
    if step > c["reset_every"]:
        prune |= np.exp(p["scales"]).max(-1) > c["prune_scale3d"] * scene_scale
        if rad is not None:
            prune |= rad > c["prune_scale2d"]
    keep = np.nonzero(~prune)[0]
    for k in p:
        p[k] = p[k][keep]
        m[k] = tuple(a[keep] for a in m[k])
    return p, m, (n_dupli, n_split, int(prune.sum()))


def reset_opacity(params, moments, value):
    """reset_opa (ops.py:214-243): clamp the opacity logits to logit(value),
    zero the opacity moments."""
    lim = float(np.log(f32(value) / (f32(1.0) - f32(value))))
    params = dict(params)
    moments = dict(moments)
    params["opacities"] = np.minimum(params["opacities"], f32(lim)).astype(f32)
    moments["opacities"] = tuple(np.zeros_like(a) for a in moments["opacities"])
    return params, moments
