"""Histogram of contributing lanes per (record, wave) in the 16x16 backward on
the bench workload (gsplat_hip_debug_set_lane_histogram); profiling aid."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from gsplat_hip import _lib
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene
    grid, W, H, _ = bench.CONFIGS["m2"]
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=grid)
    vm_pool, K_pool = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device="cuda")
    for it in range(3):
        tr.step(it)
    hist = torch.zeros(65, dtype=torch.int64, device="cuda")
    _lib.call("gsplat_hip_debug_set_lane_histogram", hist.data_ptr())
    tr.step(3)
    torch.cuda.synchronize()
    _lib.call("gsplat_hip_debug_set_lane_histogram", None)
    h = hist.cpu().tolist()
    tot = sum(h)
    cum = 0
    print(f"records x waves composited: {tot}")
    for k, v in enumerate(h):
        cum += v
        if v:
            print(f"{k:3d} {v:10d} {100 * v / tot:6.2f}% cum {100 * cum / tot:6.2f}%")


if __name__ == "__main__":
    main()
