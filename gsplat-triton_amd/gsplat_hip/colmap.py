"""COLMAP scenes for the trainer counterpart.

The reference trainer reads its scenes with `pycolmap.SceneManager`
(examples/datasets/colmap.py:59-333, a git-URL dependency pinned in
examples/requirements.txt:4 and absent here) and normalises the world with
examples/datasets/normalize.py.  This module restates both on numpy:

  read_model(dir)    cameras / images / points3D from COLMAP's binary
                     (`*.bin`) or text (`*.txt`) model files, in the formats
                     COLMAP documents (src/colmap/scene/reconstruction_io)
  similarity_from_cameras, align_principle_axes, transform_points,
  transform_cameras  normalize.py:4-143, same algebra and order
  Parser             colmap.py:59-333: world-to-camera matrices from the
                     image quaternions, K / factor per camera, images sorted
                     by name, optional normalisation, the per-image point
                     indices, the actual-image-size K rescale and scene_scale
  Dataset            colmap.py:336-440: the every-`test_every`-th split and
                     the per-item dict (K, camtoworld, image, image_id)

Undistortion of non-pinhole cameras needs OpenCV (`cv2.remap`), which this
image does not ship: the parameters are parsed and kept, and `Dataset`
raises for a distorted camera instead of returning distorted pixels.
"""

import os
import struct
from typing import Dict, List, Optional

import numpy as np

# model id -> (name, number of parameters)  (COLMAP's camera models)
CAMERA_MODELS = {
    0: ("SIMPLE_PINHOLE", 3), 1: ("PINHOLE", 4), 2: ("SIMPLE_RADIAL", 4), 3: ("RADIAL", 5),
    4: ("OPENCV", 8), 5: ("OPENCV_FISHEYE", 8), 6: ("FULL_OPENCV", 12), 7: ("FOV", 5),
    8: ("SIMPLE_RADIAL_FISHEYE", 4), 9: ("RADIAL_FISHEYE", 5), 10: ("THIN_PRISM_FISHEYE", 12),
}
MODEL_IDS = {name: i for i, (name, _) in CAMERA_MODELS.items()}


class Camera:
    def __init__(self, camera_id, model, width, height, params):
        self.id, self.model = int(camera_id), str(model)
        self.width, self.height = int(width), int(height)
        self.params = np.asarray(params, dtype=np.float64)

    def intrinsics(self):
        """(fx, fy, cx, cy) as pycolmap's Camera exposes them."""
        p, m = self.params, self.model
        if m in ("SIMPLE_PINHOLE", "SIMPLE_RADIAL", "RADIAL", "SIMPLE_RADIAL_FISHEYE",
                 "RADIAL_FISHEYE", "FOV"):
            return p[0], p[0], p[1], p[2]
        return p[0], p[1], p[2], p[3]

    def distortion(self):
        """[k1, k2, p1|k3, p2|k4] as colmap.py:111-129 builds them; empty for
        pinhole cameras."""
        p, m = self.params, self.model
        if m in ("SIMPLE_PINHOLE", "PINHOLE"):
            return np.empty(0, np.float32)
        if m == "SIMPLE_RADIAL":
            return np.array([p[3], 0, 0, 0], np.float32)
        if m == "RADIAL":
            return np.array([p[3], p[4], 0, 0], np.float32)
        if m in ("OPENCV", "OPENCV_FISHEYE"):
            return np.array(p[4:8], np.float32)
        raise NotImplementedError(f"camera model {m} (colmap.py:111-133 supports models 0-5)")


class Image:
    def __init__(self, image_id, qvec, tvec, camera_id, name, xys, point3D_ids):
        self.id, self.camera_id, self.name = int(image_id), int(camera_id), str(name)
        self.qvec = np.asarray(qvec, np.float64)  # (w, x, y, z), world -> camera
        self.tvec = np.asarray(tvec, np.float64)
        self.xys = np.asarray(xys, np.float64).reshape(-1, 2)
        self.point3D_ids = np.asarray(point3D_ids, np.int64)

    def R(self):
        w, x, y, z = self.qvec
        return np.array([
            [1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * z * x + 2 * w * y],
            [2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x],
            [2 * z * x - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y]])


class Point3D:
    def __init__(self, point_id, xyz, rgb, error, image_ids, point2D_idxs):
        self.id = int(point_id)
        self.xyz = np.asarray(xyz, np.float64)
        self.rgb = np.asarray(rgb, np.uint8)
        self.error = float(error)
        self.image_ids = np.asarray(image_ids, np.int64)
        self.point2D_idxs = np.asarray(point2D_idxs, np.int64)


# ----------------------------------------------------------------- readers
def _read(f, fmt):
    n = struct.calcsize(fmt)
    return struct.unpack(fmt, f.read(n))


def _read_cameras_bin(path):
    cams = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "<Q")
        for _ in range(n):
            cid, mid, w, h = _read(f, "<iiQQ")
            name, npar = CAMERA_MODELS[mid]
            cams[cid] = Camera(cid, name, w, h, _read(f, "<" + "d" * npar))
    return cams


def _read_images_bin(path):
    ims = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "<Q")
        for _ in range(n):
            iid, qw, qx, qy, qz, tx, ty, tz, cid = _read(f, "<idddddddi")
            name = b""
            while True:
                ch = f.read(1)
                if ch in (b"\x00", b""):
                    break
                name += ch
            (n2,) = _read(f, "<Q")
            data = np.frombuffer(f.read(24 * n2), dtype=np.dtype([("x", "<f8"), ("y", "<f8"),
                                                                  ("p", "<i8")]))
            ims[iid] = Image(iid, (qw, qx, qy, qz), (tx, ty, tz), cid, name.decode(),
                             np.stack([data["x"], data["y"]], -1), data["p"])
    return ims


def _read_points_bin(path):
    pts = {}
    with open(path, "rb") as f:
        (n,) = _read(f, "<Q")
        for _ in range(n):
            pid, x, y, z, r, g, b, err, tl = _read(f, "<QdddBBBdQ")
            track = np.frombuffer(f.read(8 * tl), dtype="<i4").reshape(-1, 2)
            pts[pid] = Point3D(pid, (x, y, z), (r, g, b), err, track[:, 0], track[:, 1])
    return pts


def _lines(path):
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                yield line


def _read_cameras_txt(path):
    cams = {}
    for line in _lines(path):
        el = line.split()
        cid, model, w, h = int(el[0]), el[1], int(el[2]), int(el[3])
        cams[cid] = Camera(cid, model, w, h, [float(x) for x in el[4:]])
    return cams


def _read_images_txt(path):
    # two lines per image; the second (its 2D points) may be empty
    with open(path) as f:
        rows = [ln.rstrip("\n") for ln in f if not ln.startswith("#")]
    while rows and not rows[-1].strip() and len(rows) % 2:
        rows.pop()
    ims = {}
    for k in range(0, len(rows) - 1, 2):
        el = rows[k].split()
        if not el:
            continue
        iid = int(el[0])
        q = [float(x) for x in el[1:5]]
        t = [float(x) for x in el[5:8]]
        cid, name = int(el[8]), " ".join(el[9:])
        pts = rows[k + 1].split()
        xys = np.array([[float(pts[i]), float(pts[i + 1])] for i in range(0, len(pts), 3)])
        ids = np.array([int(pts[i + 2]) for i in range(0, len(pts), 3)], np.int64)
        ims[iid] = Image(iid, q, t, cid, name, xys.reshape(-1, 2), ids)
    return ims


def _read_points_txt(path):
    pts = {}
    for line in _lines(path):
        el = line.split()
        pid = int(el[0])
        track = np.array([int(x) for x in el[8:]], np.int64).reshape(-1, 2)
        pts[pid] = Point3D(pid, [float(x) for x in el[1:4]], [int(x) for x in el[4:7]],
                           float(el[7]), track[:, 0], track[:, 1])
    return pts


def read_model(path: str):
    """(cameras, images, points3D) dicts keyed by id, from `path`'s
    cameras/images/points3D .bin files (or .txt when no .bin exists)."""
    if os.path.exists(os.path.join(path, "cameras.bin")):
        return (_read_cameras_bin(os.path.join(path, "cameras.bin")),
                _read_images_bin(os.path.join(path, "images.bin")),
                _read_points_bin(os.path.join(path, "points3D.bin")))
    return (_read_cameras_txt(os.path.join(path, "cameras.txt")),
            _read_images_txt(os.path.join(path, "images.txt")),
            _read_points_txt(os.path.join(path, "points3D.txt")))


def write_model_bin(path: str, cameras, images, points3D):
    """COLMAP binary model writer (the inverse of read_model; tests and tools)."""
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "cameras.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(cameras)))
        for c in cameras.values():
            f.write(struct.pack("<iiQQ", c.id, MODEL_IDS[c.model], c.width, c.height))
            f.write(struct.pack("<" + "d" * len(c.params), *c.params))
    with open(os.path.join(path, "images.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(images)))
        for im in images.values():
            f.write(struct.pack("<idddddddi", im.id, *im.qvec, *im.tvec, im.camera_id))
            f.write(im.name.encode() + b"\x00")
            f.write(struct.pack("<Q", len(im.point3D_ids)))
            for (x, y), p in zip(im.xys, im.point3D_ids):
                f.write(struct.pack("<ddq", x, y, p))
    with open(os.path.join(path, "points3D.bin"), "wb") as f:
        f.write(struct.pack("<Q", len(points3D)))
        for p in points3D.values():
            f.write(struct.pack("<QdddBBBdQ", p.id, *p.xyz, *[int(v) for v in p.rgb], p.error,
                                len(p.image_ids)))
            for i, j in zip(p.image_ids, p.point2D_idxs):
                f.write(struct.pack("<ii", i, j))


# ----------------------------------------------------------- normalisation
def _skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def similarity_from_cameras(c2w, strict_scaling=False, center_method="focus"):
    """normalize.py:4-69 restated: rotate the world so the cameras' mean up
    direction (their -y axes) becomes (0, -1, 0), recentre on the median of
    the points nearest the origin along the cameras' optical axes ("focus")
    or on the median camera position ("poses"), and scale so the median (max
    with strict_scaling) camera distance is 1."""
    pos, rot = c2w[:, :3, 3], c2w[:, :3, :3]
    cam_up = np.array([0.0, -1.0, 0.0])
    up = (-rot[:, :, 1]).mean(axis=0)  # each camera's -y axis in world space
    up = up / np.linalg.norm(up)
    cos = float(cam_up @ up)
    if cos > -1:  # Rodrigues rotation taking `up` onto cam_up
        k = _skew(np.cross(up, cam_up))
        r_align = np.eye(3) + k + (k @ k) / (1 + cos)
    else:  # exactly opposite: half turn about x
        r_align = np.diag([-1.0, 1.0, 1.0])
    axes = (r_align @ rot)[:, :, 2]  # optical axes after the rotation
    pos = pos @ r_align.T
    if center_method == "focus":
        foot = pos - (axes * pos).sum(-1, keepdims=True) * axes
        shift = -np.median(foot, axis=0)
    elif center_method == "poses":
        shift = -np.median(pos, axis=0)
    else:
        raise ValueError(f"Unknown center_method {center_method}")
    dist = np.linalg.norm(pos + shift, axis=-1)
    scale = 1.0 / (dist.max() if strict_scaling else np.median(dist))
    out = np.eye(4)
    out[:3, :3] = r_align * scale
    out[:3, 3] = shift * scale
    return out


def align_principle_axes(point_cloud):
    """normalize.py:72-104 restated: a rigid transform to the median-centred
    principal axes of the points, the largest variance on x and the smallest
    on z, kept right-handed."""
    centre = np.median(point_cloud, axis=0)
    evals, evecs = np.linalg.eigh(np.cov(point_cloud - centre, rowvar=False))
    basis = evecs[:, np.argsort(evals)[::-1]]
    if np.linalg.det(basis) < 0:
        basis[:, 0] = -basis[:, 0]
    out = np.eye(4)
    out[:3, :3] = basis.T
    out[:3, 3] = -basis.T @ centre
    return out


def transform_points(matrix, points):
    """normalize.py:107-119: x -> A x + b for an affine 4x4."""
    assert matrix.shape == (4, 4) and points.ndim == 2 and points.shape[1] == 3
    return points @ matrix[:3, :3].T + matrix[:3, 3]


def transform_cameras(matrix, camtoworlds):
    """normalize.py:122-136: left-multiply every camera-to-world matrix by the
    similarity, then divide the scale back out of the rotation block."""
    assert matrix.shape == (4, 4) and camtoworlds.ndim == 3 and camtoworlds.shape[1:] == (4, 4)
    out = matrix[None] @ camtoworlds
    norm = np.linalg.norm(out[:, 0, :3], axis=1)
    out[:, :3, :3] /= norm[:, None, None]
    return out


def _rel_paths(d):
    out = []
    for dp, _, fn in os.walk(d):
        out += [os.path.relpath(os.path.join(dp, f), d) for f in fn]
    return out


# ------------------------------------------------------------------ parser
class Parser:
    """colmap.py:59-333 on read_model (no pycolmap, no OpenCV)."""

    def __init__(self, data_dir: str, factor: int = 1, normalize: bool = False,
                 test_every: int = 8):
        self.data_dir, self.factor = data_dir, factor
        self.normalize, self.test_every = normalize, test_every
        colmap_dir = os.path.join(data_dir, "sparse/0/")
        if not os.path.exists(colmap_dir):
            colmap_dir = os.path.join(data_dir, "sparse")
        assert os.path.exists(colmap_dir), f"COLMAP directory {colmap_dir} does not exist."
        cameras, images, points3D = read_model(colmap_dir)
        if len(images) == 0:
            raise ValueError("No images found in COLMAP.")

        bottom = np.array([0, 0, 0, 1.0]).reshape(1, 4)
        w2c, camera_ids, names = [], [], []
        Ks, params, imsize, masks = {}, {}, {}, {}
        for k in images:  # the model's order, then sorted by name below
            im = images[k]
            w2c.append(np.concatenate([np.concatenate([im.R(), im.tvec.reshape(3, 1)], 1),
                                       bottom], 0))
            camera_ids.append(im.camera_id)
            names.append(im.name)
            cam = cameras[im.camera_id]
            fx, fy, cx, cy = cam.intrinsics()
            K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
            K[:2, :] /= factor
            Ks[im.camera_id] = K
            params[im.camera_id] = cam.distortion()
            imsize[im.camera_id] = (cam.width // factor, cam.height // factor)
            masks[im.camera_id] = None
        camtoworlds = np.linalg.inv(np.stack(w2c, 0))
        inds = np.argsort(names)
        names = [names[i] for i in inds]
        camtoworlds = camtoworlds[inds]
        camera_ids = [camera_ids[i] for i in inds]

        # images (the `images_<factor>` folder mapped to COLMAP's by sorted order)
        suffix = f"_{factor}" if factor > 1 else ""
        colmap_image_dir = os.path.join(data_dir, "images")
        image_dir = os.path.join(data_dir, "images" + suffix)
        self.image_paths = []
        if os.path.exists(image_dir) and os.path.exists(colmap_image_dir):
            mapping = dict(zip(sorted(_rel_paths(colmap_image_dir)),
                               sorted(_rel_paths(image_dir))))
            self.image_paths = [os.path.join(image_dir, mapping[n]) for n in names]

        ordered = sorted(points3D)
        idx_of = {pid: i for i, pid in enumerate(ordered)}
        points = np.array([points3D[p].xyz for p in ordered], np.float32).reshape(-1, 3)
        points_err = np.array([points3D[p].error for p in ordered], np.float32)
        points_rgb = np.array([points3D[p].rgb for p in ordered], np.uint8).reshape(-1, 3)
        name_of = {im.id: im.name for im in images.values()}
        point_indices: Dict[str, List[int]] = {}
        for p in ordered:
            for iid in points3D[p].image_ids:
                point_indices.setdefault(name_of[int(iid)], []).append(idx_of[p])
        self.point_indices = {k: np.array(v, np.int32) for k, v in point_indices.items()}

        if normalize:
            T1 = similarity_from_cameras(camtoworlds)
            camtoworlds = transform_cameras(T1, camtoworlds)
            points = transform_points(T1, points)
            T2 = align_principle_axes(points)
            camtoworlds = transform_cameras(T2, camtoworlds)
            points = transform_points(T2, points)
            transform = T2 @ T1
        else:
            transform = np.eye(4)

        self.image_names, self.camtoworlds, self.camera_ids = names, camtoworlds, camera_ids
        self.Ks_dict, self.params_dict, self.imsize_dict = Ks, params, imsize
        self.mask_dict = masks
        self.points, self.points_err, self.points_rgb = points, points_err, points_rgb
        self.transform = transform

        # actual image size vs COLMAP's (colmap.py:237-247)
        if self.image_paths:
            from PIL import Image as PILImage
            with PILImage.open(self.image_paths[0]) as img:
                aw, ah = img.size
            cw, ch = self.imsize_dict[self.camera_ids[0]]
            sw, sh = aw / cw, ah / ch
            for cid, K in self.Ks_dict.items():
                K[0, :] *= sw
                K[1, :] *= sh
                w, h = self.imsize_dict[cid]
                self.imsize_dict[cid] = (int(w * sw), int(h * sh))

        locs = camtoworlds[:, :3, 3]
        self.scene_scale = float(np.max(np.linalg.norm(locs - locs.mean(0), axis=1)))


class Dataset:
    """colmap.py:336-440: every `test_every`-th image is a test image."""

    def __init__(self, parser: Parser, split: str = "train", patch_size: Optional[int] = None):
        self.parser, self.split, self.patch_size = parser, split, patch_size
        idx = np.arange(len(parser.image_names))
        self.indices = idx[idx % parser.test_every != 0] if split == "train" else \
            idx[idx % parser.test_every == 0]

    def __len__(self):
        return len(self.indices)

    def __getitem__(self, item: int):
        import torch
        from PIL import Image as PILImage
        index = self.indices[item]
        cid = self.parser.camera_ids[index]
        if len(self.parser.params_dict[cid]) > 0:
            raise NotImplementedError("undistortion of a non-pinhole COLMAP camera needs "
                                      "OpenCV's remap (colmap.py:364-372), not in this image")
        with PILImage.open(self.parser.image_paths[index]) as img:
            image = np.array(img.convert("RGB"))
        K = self.parser.Ks_dict[cid].copy()
        if self.patch_size is not None:
            h, w = image.shape[:2]
            x = np.random.randint(0, max(w - self.patch_size, 1))
            y = np.random.randint(0, max(h - self.patch_size, 1))
            image = image[y:y + self.patch_size, x:x + self.patch_size]
            K[0, 2] -= x
            K[1, 2] -= y
        return {"K": torch.from_numpy(K).float(),
                "camtoworld": torch.from_numpy(self.parser.camtoworlds[index]).float(),
                "image": torch.from_numpy(np.ascontiguousarray(image)).float(),
                "image_id": item}
