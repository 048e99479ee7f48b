"""COLMAP scene layer of the trainer counterpart (gsplat_hip.colmap; SURVEY
§8 f1, replacing pycolmap + examples/datasets/normalize.py).

* normalisation: pinned to the reference's own normalize.py run on numpy
  (tests/golden/make_golden_colmap.py -> colmap_normalize.npz);
* model files: binary round trip through write_model_bin / read_model, the
  text format parsed to the same values, and Parser / Dataset on a synthetic
  scene (sorted image names, K / factor, point indices, scene_scale)."""

import os

import numpy as np
import pytest

from conftest import load_golden


def test_normalize_matches_reference():
    from gsplat_hip import colmap as M
    g = load_golden("colmap_normalize")
    np.testing.assert_allclose(M.similarity_from_cameras(g["c2w"]), g["T1"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(M.similarity_from_cameras(g["c2w"], strict_scaling=True),
                               g["T1_strict"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(M.similarity_from_cameras(g["c2w"], center_method="poses"),
                               g["T1_poses"], rtol=0, atol=1e-12)
    c1 = M.transform_cameras(g["T1"], g["c2w"].copy())
    np.testing.assert_allclose(c1, g["c1"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(M.transform_points(g["T1"], g["pts"]), g["p1"], rtol=0, atol=1e-12)
    T2 = M.align_principle_axes(g["p1"])
    np.testing.assert_allclose(T2, g["T2"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(M.transform_cameras(g["T2"], g["c1"].copy()), g["c2"], rtol=0,
                               atol=1e-12)


def _scene(tmp, n_img=5, n_pts=40, seed=0):
    from gsplat_hip import colmap as M
    rng = np.random.default_rng(seed)
    cams = {1: M.Camera(1, "PINHOLE", 640, 480, [500.0, 510.0, 320.0, 240.0]),
            2: M.Camera(2, "SIMPLE_PINHOLE", 320, 240, [250.0, 160.0, 120.0])}
    ims = {}
    for i in range(1, n_img + 1):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        ids = rng.choice(np.arange(1, n_pts + 1), size=6, replace=False)
        ims[i] = M.Image(i, q, rng.normal(size=3), 1 + (i % 2), f"img_{(n_img - i):03d}.png",
                         rng.random((6, 2)) * 100, ids)
    pts = {}
    for p in range(1, n_pts + 1):
        seen = [i for i, im in ims.items() if p in im.point3D_ids]
        pts[p] = M.Point3D(p, rng.normal(size=3), rng.integers(0, 255, 3), rng.random(),
                           seen, [list(ims[i].point3D_ids).index(p) for i in seen])
    return cams, ims, pts


def _write_txt(path, cams, ims, pts):
    def fl(v):
        return " ".join(repr(float(x)) for x in v)
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "cameras.txt"), "w") as f:
        f.write("# Camera list\n")
        for c in cams.values():
            f.write(f"{c.id} {c.model} {c.width} {c.height} " + fl(c.params) + "\n")
    with open(os.path.join(path, "images.txt"), "w") as f:
        f.write("# Image list\n")
        for im in ims.values():
            f.write(f"{im.id} " + fl(im.qvec) + " " + fl(im.tvec)
                    + f" {im.camera_id} {im.name}\n")
            f.write(" ".join(f"{float(x)!r} {float(y)!r} {p}" for (x, y), p in zip(im.xys, im.point3D_ids))
                    + "\n")
    with open(os.path.join(path, "points3D.txt"), "w") as f:
        for p in pts.values():
            track = " ".join(f"{i} {j}" for i, j in zip(p.image_ids, p.point2D_idxs))
            f.write(f"{p.id} " + fl(p.xyz) + " " + " ".join(str(int(v)) for v in p.rgb)
                    + f" {float(p.error)!r} {track}\n")


@pytest.mark.parametrize("fmt", ["bin", "txt"])
def test_model_round_trip(tmp_path, fmt):
    from gsplat_hip import colmap as M
    cams, ims, pts = _scene(tmp_path)
    d = str(tmp_path / "sparse" / "0")
    if fmt == "bin":
        M.write_model_bin(d, cams, ims, pts)
    else:
        _write_txt(d, cams, ims, pts)
    c2, i2, p2 = M.read_model(d)
    assert sorted(c2) == sorted(cams) and sorted(i2) == sorted(ims) and sorted(p2) == sorted(pts)
    for k, c in cams.items():
        assert (c2[k].model, c2[k].width, c2[k].height) == (c.model, c.width, c.height)
        np.testing.assert_array_equal(c2[k].params, c.params)
    for k, im in ims.items():
        assert i2[k].name == im.name and i2[k].camera_id == im.camera_id
        np.testing.assert_array_equal(i2[k].qvec, im.qvec)
        np.testing.assert_array_equal(i2[k].tvec, im.tvec)
        np.testing.assert_array_equal(i2[k].xys, im.xys)
        np.testing.assert_array_equal(i2[k].point3D_ids, im.point3D_ids)
        R = i2[k].R()
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)
    for k, p in pts.items():
        np.testing.assert_array_equal(p2[k].xyz, p.xyz)
        np.testing.assert_array_equal(p2[k].rgb, p.rgb)
        np.testing.assert_array_equal(p2[k].image_ids, p.image_ids)


@pytest.mark.parametrize("normalize", [False, True])
def test_parser_and_dataset(tmp_path, normalize):
    from PIL import Image as PILImage
    from gsplat_hip import colmap as M
    cams, ims, pts = _scene(tmp_path, n_img=10)
    M.write_model_bin(str(tmp_path / "sparse" / "0"), cams, ims, pts)
    factor = 2
    for sub, div in (("images", 1), ("images_2", 2)):
        os.makedirs(tmp_path / sub, exist_ok=True)
        for im in ims.values():
            c = cams[im.camera_id]
            PILImage.new("RGB", (c.width // div, c.height // div), (10, 20, 30)).save(
                tmp_path / sub / im.name)
    P = M.Parser(str(tmp_path), factor=factor, normalize=normalize, test_every=4)
    assert P.image_names == sorted(im.name for im in ims.values())
    by_name = {im.name: im for im in ims.values()}
    for n, c2w, cid in zip(P.image_names, P.camera_ids, P.camera_ids):
        assert cid == by_name[n].camera_id
    if not normalize:
        for n, c2w in zip(P.image_names, P.camtoworlds):
            im = by_name[n]
            w2c = np.eye(4)
            w2c[:3, :3], w2c[:3, 3] = im.R(), im.tvec
            np.testing.assert_allclose(c2w, np.linalg.inv(w2c), atol=1e-12)
    fx, fy, cx, cy = cams[1].intrinsics()
    np.testing.assert_allclose(P.Ks_dict[1], [[fx / 2, 0, cx / 2], [0, fy / 2, cy / 2], [0, 0, 1]])
    # images of the first camera sized as COLMAP / factor: no rescale
    assert P.imsize_dict[1] == (320, 240)
    assert P.points.shape == (len(pts), 3) and P.points_rgb.shape == (len(pts), 3)
    for n, idx in P.point_indices.items():  # every image observes 6 points
        assert len(idx) == 6 and idx.max() < len(pts)
    locs = P.camtoworlds[:, :3, 3]
    assert P.scene_scale == pytest.approx(np.max(np.linalg.norm(locs - locs.mean(0), axis=1)))
    tr, te = M.Dataset(P, "train"), M.Dataset(P, "val")
    assert len(tr) + len(te) == 10 and list(te.indices) == [0, 4, 8]
    item = tr[0]
    assert item["image"].shape[-1] == 3 and item["K"].shape == (3, 3)
    assert item["camtoworld"].shape == (4, 4)
