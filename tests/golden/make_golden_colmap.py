"""Golden vectors for the COLMAP scene normalisation (gsplat_hip.colmap)
from the REFERENCE's examples/datasets/normalize.py, run here on numpy.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden_colmap.py

Loads normalize.py by path (it imports numpy only) and stores inputs and
outputs as colmap_normalize.npz next to this script.
"""

import importlib.util
import os

import numpy as np

REF = "/root/reference/examples/datasets/normalize.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "colmap_normalize.npz")


def rand_cameras(rng, n):
    """Cameras on a noisy ring looking at the origin, OpenCV convention."""
    c2w = np.tile(np.eye(4), (n, 1, 1))
    for i in range(n):
        a = 2 * np.pi * i / n
        pos = np.array([4 * np.cos(a), 4 * np.sin(a), 1.5]) + rng.normal(0, 0.2, 3)
        fwd = -pos / np.linalg.norm(pos) + rng.normal(0, 0.05, 3)
        fwd /= np.linalg.norm(fwd)
        right = np.cross(fwd, np.array([0, 0, 1.0]))
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        c2w[i, :3, :3] = np.stack([right, down, fwd], 1)
        c2w[i, :3, 3] = pos
    return c2w


def main():
    spec = importlib.util.spec_from_file_location("ref_normalize", REF)
    N = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(N)
    rng = np.random.default_rng(0)
    c2w = rand_cameras(rng, 24)
    pts = rng.normal(0, 1, (500, 3)) * [2.0, 1.0, 0.3] + [0.3, -0.2, 0.1]
    T1 = N.similarity_from_cameras(c2w)
    T1s = N.similarity_from_cameras(c2w, strict_scaling=True)
    T1p = N.similarity_from_cameras(c2w, center_method="poses")
    c1 = N.transform_cameras(T1, c2w.copy())
    p1 = N.transform_points(T1, pts)
    T2 = N.align_principle_axes(p1)
    c2 = N.transform_cameras(T2, c1.copy())
    p2 = N.transform_points(T2, p1)
    np.savez_compressed(OUT, c2w=c2w, pts=pts, T1=T1, T1_strict=T1s, T1_poses=T1p, c1=c1, p1=p1,
                        T2=T2, c2=c2, p2=p2)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
