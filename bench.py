"""Benchmark: 3DGS train-step images/sec on garden-like M2 (1,006,065
Gaussians, 1920x1080, SH degree 3), per-camera data parallel over N GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config m2|m3|m1]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = render one camera per rank through the HIP hot path (projection,
SH, isect + sort, rasterize), 0.8*L1 + 0.2*(1-SSIM) loss, backward, RCCL
all-reduce of the Gaussian gradients (N > 1), DefaultStrategy statistics and
Adam (see gsplat_hip/train_step.py).  Inputs are resident in HBM.

Rank 0 prints one JSON line with the driver's contract plus
  roofline:     rasterize_to_pixels fwd -- algorithmic bytes per launch /
                mean HIP-event duration of that launch in the timed region
  cpu_baseline: the numpy oracle's train step on the host (bounded sample).
"""

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gsplat-triton_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
CONFIGS = {
    # name: (scene_grid, width, height, description)
    "m2": (3, 1920, 1080, "garden scene_grid=3 (1,006,065 Gaussians), 1920x1080, SH deg 3"),
    "m3": (7, 1920, 1080, "garden scene_grid=7 (5,477,465 Gaussians), 1920x1080, SH deg 3"),
    "m1": (1, 648, 420, "garden crop (111,785 Gaussians), 648x420, SH deg 3"),
    # BASELINE.json configs[4]: the 2DGS surfel pipeline on the M2 scene
    "m5": (3, 1920, 1080, "2DGS surfels (simple_trainer_2dgs default step, RGB+D), garden "
                          "scene_grid=3 (1,006,065 surfels), 1920x1080, SH deg 3"),
}
MODEL = {"m5": "2dgs"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="m2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-tile-stride", type=int, default=24)
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 PMC child runs that measure roofline.traffic")
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def pmc_traffic(config: str):
    """HBM bytes of one rasterize-forward launch from rocprofv3 counters.

    Two child runs of `bench.py --probe` under rocprofv3 (separate --pmc
    passes: FETCH_SIZE and WRITE_SIZE cannot share one), started before this
    process touches the GPU.  Corrections per MI355X_MICROARCH.md "HBM":
    FETCH_SIZE is in KiB and counts half the bytes on gfx950 (x2);
    WRITE_SIZE is in KiB.  Returns None when rocprofv3 is unavailable."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(rp):
        return None
    if any("rocprof" in v.lower() for k, v in os.environ.items() if k in ("LD_PRELOAD", "HSA_TOOLS_LIB")) \
            or any(k.startswith("ROCPROF") for k in os.environ):
        return None  # already running under a profiler: no nested profiler runs
    env = dict(os.environ, TMPDIR="/tmp")
    per = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"):
        d = tempfile.mkdtemp(prefix="gsplat_pmc_", dir="/tmp")
        regex = "surfel::fwd2?_kernel" if MODEL.get(config) == "2dgs" else "r16::fwd2?_kernel"
        cmd = [rp, "--kernel-include-regex", regex, "--pmc", ctr, "-f", "csv",
               "-d", d, "-o", "p", "--", sys.executable, os.path.abspath(__file__), "--probe",
               "--config", config, "--warmup", "2"]
        try:
            subprocess.run(cmd, env=env, cwd="/tmp", timeout=300, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except (subprocess.SubprocessError, OSError):
            return None
        vals = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == ctr:
                    vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        shutil.rmtree(d, ignore_errors=True)
        if not vals:
            if ctr == "SQ_INSTS_VALU":  # optional: VALU issue rate of the same launch
                continue
            return None
        per[ctr] = float(np.mean(list(vals.values())))
    fetch = 2.0 * per["FETCH_SIZE"] * 1024.0
    write = per["WRITE_SIZE"] * 1024.0
    return {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
            "fetch_size_kib": per["FETCH_SIZE"], "write_size_kib": per["WRITE_SIZE"],
            "valu_insts": per.get("SQ_INSTS_VALU"),
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --probe "
                      "(FETCH_SIZE x2 per MI355X_MICROARCH.md; gathers uncalibrated)"}


def _valu_frac(traffic, launch_ms):
    if not traffic or not traffic.get("valu_insts") or not launch_ms == launch_ms:
        return None
    insts = traffic["valu_insts"]
    peak = 1024 * 2.4e9 / 2.0  # wave64 VALU instructions per second, whole chip
    achieved = insts / (launch_ms * 1e-3)
    return {"bound": "valu", "insts_per_launch": insts, "achieved": achieved, "peak": peak,
            "unit": "wave-instr/s", "frac": achieved / peak}


def max_over_ranks(elapsed: float, world: int, device) -> float:
    """The job's time: the slowest rank's (all_reduce MAX; identity at N=1)."""
    if world == 1:
        return elapsed
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    traffic = None
    if rank == 0 and world == 1 and not args.no_traffic and not args.probe:
        traffic = pmc_traffic(args.config)  # child processes, before this one uses the GPU
    dev = f"cuda:{local}"
    torch.cuda.set_device(dev)

    import gsplat_hip  # noqa: F401  (raises if libgsplat_hip.so is missing)
    from gsplat_hip import _wrapper
    from gsplat_hip.train_step import Trainer, camera_pool, load_garden_scene

    grid, W, H, desc = CONFIGS[args.config]
    means, rgbs, vms, Ks, sw, sh_ = load_garden_scene(
        os.path.join(ROOT, "tests", "golden", "garden_scene.npz"), scene_grid=grid)
    vm_pool, K_pool = camera_pool(vms, Ks, sw, sh_, W, H, n=max(8, world))
    model = MODEL.get(args.config, "3dgs")
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device=dev, world_size=world,
                 rank=rank, model=model)
    N = means.shape[0]

    for it in range(args.warmup):
        tr.step(it)
    torch.cuda.synchronize()
    if args.probe:  # PMC child run: a few steps, no output
        for it in range(args.warmup, args.warmup + 2):
            tr.step(it)
        torch.cuda.synchronize()
        return

    timers = _wrapper.enable_kernel_timers(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(args.warmup, args.warmup + args.steps):
        tr.step(it)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    _wrapper.enable_kernel_timers(False)

    # ---- per-kernel HIP-event times over the timed region
    def mean_ms(name):
        evs = timers.get(name, [])
        return float(np.mean([a.elapsed_time(b) for a, b in evs])) if evs else float("nan")

    two = model == "2dgs"
    kname = "rasterize_2dgs_fwd" if two else "rasterize_fwd"
    fwd_ms, bwd_ms = mean_ms(kname), mean_ms("rasterize_2dgs_bwd" if two else "rasterize_bwd")

    # ---- algorithmic bytes of one rasterize fwd launch, averaged over the
    # cameras this rank renders (computed outside the timed region).
    # 3DGS: per isect id 4 + means2d 8 + conic 12 + opacity 4 + colour 4D,
    #       per pixel colour 4D + alpha 4 + last id 4.
    # 2DGS: per isect id 4 + means2d 8 + ray transform 36 + opacity 4 +
    #       normal 12 + colour 4D; per pixel colour 4D + alpha, normal (12),
    #       distortion, median, last id, median id.
    D = 4 if two else 3
    per_isect = (64 + 4 * D) if two else (28 + 4 * D)
    per_px = (4 * D + 32) if two else (4 * D + 8)
    node_name = "_RasterizeToPixels2DGSBackward" if two else "_RasterizeToPixelsBackward"
    last_slot = 12 if two else 9
    byts, isects = [], []
    if True:  # graph needed to reach the forward's saved last_ids
        for it in range(args.warmup, args.warmup + min(args.steps, len(vm_pool))):
            ci = tr.camera_index(it)
            colors, alphas, meta = tr.render(ci)
            # last_ids are internal to the autograd node; recompute n_eff from
            # the forward outputs with the same kernel
            offs = meta["isect_offsets"].flatten().long()
            n = meta["flatten_ids"].numel()
            ends = torch.cat([offs[1:], torch.tensor([n], device=dev)])
            node = colors.grad_fn
            while node is not None and type(node).__name__ != node_name:
                node = node.next_functions[0][0]
            last = node.saved_tensors[last_slot] if node is not None else None
            if last is not None:
                ts = meta["tile_size"]
                tw, th = meta["tile_width"], meta["tile_height"]
                lp = torch.nn.functional.pad(last[0], (0, tw * ts - W, 0, th * ts - H))
                tmax = lp.view(th, ts, tw, ts).amax(dim=(1, 3)).flatten().long()
                n_eff = int(torch.clamp(torch.minimum(ends, tmax + 1) - offs, min=0).sum())
            else:
                n_eff = n
            P = H * W
            byts.append(n_eff * per_isect + P * per_px + 4 * tw * th)
            isects.append(n)
    bytes_per_launch = float(np.mean(byts))
    achieved = bytes_per_launch / (fwd_ms * 1e-3) / 1e9

    result = {
        "metric": "train-step images/sec + rasterize fwd HBM GB/s, garden 1080p, 1/2/4/8 MI355X",
        "value": world * args.steps / elapsed,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: garden SfM points (assets/test_garden.npz crop) tiled 3x3, random "
                "scales/quats/opacities, random target images",
        "config": {"workload": desc, "gaussians": N, "width": W, "height": H,
                   "cameras_per_rank_per_step": 1, "parallelism": f"dp{world}",
                   "n_isects_mean": float(np.mean(isects)), "packed": False,
                   "loss": "0.8*L1+0.2*(1-SSIM valid)", "optimizer": "Adam (6 groups)"},
        "roofline": {"kernel": kname, "bound": "hbm", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None if traffic is None else traffic["bytes_per_launch"],
                     "traffic_detail": traffic,
                     "algorithmic_bytes_per_launch": bytes_per_launch,
                     "launch_ms": fwd_ms, "rasterize_bwd_ms": bwd_ms},
        "model": model,
    }

    # the kernel's binding ceiling is VALU issue, not HBM: wave64
    # VALU instructions x 2 cycles each (MI355X_MICROARCH.md constants:
    # v_fma_f32 2 cyc per SIMD) against 1024 SIMDs x 2.4 GHz over the launch
    # time; SQ_INSTS_VALU from a rocprofv3 --pmc pass of the same workload
    result["roofline"]["valu"] = _valu_frac(traffic, fwd_ms)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(tr, args.cpu_tile_stride)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(tr, stride):
    from oracle.cpu_step import cpu_train_step
    p = {k: v.detach().cpu().numpy() for k, v in tr.params.items()}
    sh = np.concatenate([p["sh0"], p["shN"]], 1)
    ci = 0
    total, parts, sample = cpu_train_step(
        p["means"], p["quats"], p["scales"], p["opacities"], sh, tr.viewmats[ci].cpu().numpy(),
        tr.Ks[ci].cpu().numpy(), tr.width, tr.height, tr.targets[ci].cpu().numpy(),
        tile_stride=stride)
    return {"value": 1.0 / total, "unit": "images/s", "cores": 1, "kind": "port",
            "sample": sample, "seconds_per_step_estimate": total,
            "breakdown_s": {k: round(v, 3) for k, v in parts.items()},
            "host_cpus": os.cpu_count()}


if __name__ == "__main__":
    main()
