"""torch.profiler op table of one bench training step (GPU box; profiling aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    import bench
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene
    grid, W, H, _ = bench.CONFIGS["m2"]
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=grid)
    vm_pool, K_pool = camera_pool(vms, Ks, sw, sh_, W, H, n=8)
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device="cuda")
    for it in range(3):
        tr.step(it)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        for it in range(3, 5):
            tr.step(it)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(
        sort_by="self_device_time_total", row_limit=150, max_name_column_width=40,
        max_shapes_column_width=60))


if __name__ == "__main__":
    main()
