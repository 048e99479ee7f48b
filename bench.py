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
# BASELINE.json configs[2] "densification on": simple_trainer.py's default run
# (SfM init with knn scales, SH degree schedule, means ExponentialLR,
# DefaultStrategy refine/reset); the timed window is centred on a refine step
# after the SH degree has reached 3 (steps numbered from REFINE_AT - warmup -
# steps // 2)
DENSIFY = {"m3"}
REFINE_AT = 3100


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="m2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-tile-stride", type=int, default=0,
                    help="rasterize every k-th tile in the CPU baseline (0: auto)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 PMC child runs that measure roofline.traffic")
    ap.add_argument("--eager", action="store_true",
                    help="issue every launch from the host each step instead of replaying "
                         "the step captured as a HIP graph")
    ap.add_argument("--graph", action="store_true",
                    help="replay the captured step also for the densifying config (m3), whose "
                         "default is eager: each refine re-captures, and the timed window "
                         "centred on a refine ran 213.6 graph-replayed against 228.8 images/s "
                         "eager (profiles/r4_final)")
    ap.add_argument("--mcmc", action="store_true",
                    help="the densifying schedule of simple_trainer.py's mcmc preset instead "
                         "(MCMCStrategy: relocate / add every 100 steps, per-step position "
                         "noise; init opacity 0.5, init scale 0.1, opacity / scale "
                         "regularisers 0.01), timed window centred on a refine step; the "
                         "steps between refines are graph replays unless --eager")
    ap.add_argument("--dp-path", action="store_true",
                    help="replicated data parallelism instead of the default Gaussian "
                         "sharding at N>1 (every rank holds all Gaussians; sharded Adam, "
                         "early SH reduce-scatter, per-group communicators); at N=1 that "
                         "code path over a 1-rank RCCL group")
    ap.add_argument("--dp-emulate", type=int, default=0, metavar="W",
                    help="with --dp-path: shard the optimizer rows as W ranks would and "
                         "update this rank's share (the per-rank compute of a W-GPU step; "
                         "the collectives of W ranks are not executed)")
    ap.add_argument("--gshard-emulate", type=int, default=0, metavar="W",
                    help="one GPU times rank 0 of a W-rank Gaussian-sharded step: its shard, "
                         "its camera, the other ranks' exchanged rows from stand-ins "
                         "recorded from their own renders (exchanges as device copies, no "
                         "xGMI time; measurement only)")
    ap.add_argument("--no-dp-phase", action="store_true",
                    help="at N>1: skip the second timed region that runs the replicated "
                         "per-camera data-parallel scheme (north_star's) after the default "
                         "Gaussian-sharded one (config.dp)")
    ap.add_argument("--dp-phase", action="store_true",
                    help="run that data-parallel phase at N=1 too (a 1-rank RCCL group with "
                         "the collectives issued: the N>1 code path on one GPU)")
    ap.add_argument("--watchdog-s", type=float,
                    default=float(os.environ.get("GSPLAT_HIP_WATCHDOG_S", "120")),
                    help="end the job (status 3, rank / step / phase on stderr) when a rank "
                         "makes no progress for this long; also the process group's "
                         "collective timeout (0: off)")
    ap.add_argument("--debug-hang", default="", metavar="RANK:STEP", help=argparse.SUPPRESS)
    ap.add_argument("--probe", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",),
              ("SQ_INSTS_VALU", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_LDS",
               "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"),
              ("TCC_HIT_sum", "TCC_MISS_sum"))


def pmc_traffic(config: str):
    """Counters of the rasterize forward and backward launches from rocprofv3.

    One child run of `bench.py --probe` under rocprofv3 per --pmc pass
    (FETCH_SIZE and WRITE_SIZE cannot share a pass; the SQ counters share
    one), started before this process touches the GPU.  Corrections per
    MI355X_MICROARCH.md "HBM": FETCH_SIZE is in KiB and counts half the bytes
    of a wide read on gfx950 (x2); WRITE_SIZE is in KiB (exact for float
    atomics and 16-B stores).  Returns {"fwd": {...}, "bwd": {...}} or None
    when rocprofv3 is unavailable."""
    import csv
    import glob
    import re
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
    ns = "surfel" if MODEL.get(config) == "2dgs" else "r16"
    regex = f"{ns}::(fwd|bwd)2?s?_kernel"
    per = {"fwd": {}, "bwd": {}}
    for ctrs in PMC_PASSES:
        d = tempfile.mkdtemp(prefix="gsplat_pmc_", dir="/tmp")
        cmd = [rp, "--kernel-include-regex", regex, "--pmc", *ctrs, "-f", "csv",
               "-d", d, "-o", "p", "--", sys.executable, os.path.abspath(__file__), "--probe",
               "--config", config, "--warmup", "2"]
        try:
            subprocess.run(cmd, env=env, cwd="/tmp", timeout=300, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except (subprocess.SubprocessError, OSError):
            shutil.rmtree(d, ignore_errors=True)
            if ctrs[0].startswith(("SQ_", "TCC_HIT")):
                continue  # optional pass
            return None
        vals = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(rf"{ns}::(fwd|bwd)", r["Kernel_Name"])
                if m is None or r["Counter_Name"] not in ctrs:
                    continue
                key = (m.group(1), r["Counter_Name"], r["Dispatch_Id"])
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
        shutil.rmtree(d, ignore_errors=True)
        for (k, c, _), v in vals.items():
            per[k].setdefault(c, []).append(v)
    out = {}
    for k, cs in per.items():
        mean = {c: float(np.mean(v)) for c, v in cs.items()}
        if "FETCH_SIZE" not in mean or "WRITE_SIZE" not in mean:
            return None
        fetch = 2.0 * mean["FETCH_SIZE"] * 1024.0
        write = mean["WRITE_SIZE"] * 1024.0
        out[k] = {"bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                  "counters": mean}
    out["source"] = ("rocprofv3 --pmc passes of bench.py --probe: " +
                     "; ".join(",".join(p) for p in PMC_PASSES) +
                     " (FETCH_SIZE x2 per MI355X_MICROARCH.md; gathers uncalibrated)")
    return out


def _valu_frac(pmc, launch_ms):
    """VALU issue: wave64 VALU instructions x 2 cycles (a wave64 v_fma_f32
    / v_mul_f32 issues every 2.3-2.4 cycles per SIMD at the nominal 2.4 GHz,
    tools/valu_bench.hip -> profiles/r3_valu/valu_bench.txt) against 1024
    SIMDs x 2.4 GHz over the launch."""
    ctr = (pmc or {}).get("counters", {})
    insts = ctr.get("SQ_INSTS_VALU")
    if not insts or not launch_ms == launch_ms:
        return None
    peak = 1024 * 2.4e9 / 2.0  # wave64 VALU instructions per second, whole chip
    achieved = insts / (launch_ms * 1e-3)
    res = {"bound": "valu", "insts_per_launch": insts, "achieved": achieved, "peak": peak,
           "unit": "wave-instr/s", "frac": achieved / peak}
    if ctr.get("SQ_WAVE_CYCLES"):
        res["wait_inst_any_frac"] = ctr.get("SQ_WAIT_INST_ANY", 0.0) / ctr["SQ_WAVE_CYCLES"]
    if ctr.get("SQ_INSTS_SALU"):
        res["salu_per_valu"] = ctr["SQ_INSTS_SALU"] / insts
    if ctr.get("TCC_HIT_sum") is not None and ctr.get("TCC_MISS_sum") is not None:
        tot = ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"]
        res["l2_hit_rate"] = ctr["TCC_HIT_sum"] / tot if tot else None
    return res


def max_over_ranks(elapsed: float, world: int, device) -> float:
    """The job's time: the slowest rank's (all_reduce MAX; identity at N=1)."""
    if world == 1:
        return elapsed
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n: int, argv, port: int):
    """The child command that runs `n` ranks of this script, one per GPU:
    torch.distributed.run on one node, rendezvous on 127.0.0.1 (the reference's
    `cli` spawns one process per visible GPU the same way,
    gsplat/distributed.py:304-360)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def launch(n: int, argv) -> int:
    """`bench.py --gpus N` without a torchrun environment: start the N ranks as a
    CHILD process (this parent never touches the GPU and never execs), let rank
    0's JSON line through on the shared stdout, return the children's exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(launch_cmd(n, argv, _free_port()), env=env).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:]))
    # stdout carries exactly one line, rank 0's JSON: everything else written
    # to fd 1 from here on (RCCL's version banner, library prints) goes to
    # stderr.  The launcher parent above keeps its stdout for the children.
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    cpu_pool = None
    if world > 1:
        args.no_cpu_baseline = True  # the CPU baseline is an N=1 measurement
    if rank == 0 and not args.no_cpu_baseline and not args.probe:
        # the CPU baseline's worker processes start before this process
        # touches the GPU (spawned interpreters running numpy only)
        from oracle.cpu_step import CpuPool
        cpu_pool = CpuPool(host_threads())
    if args.dp_emulate:
        args.dp_path = True
        assert world == 1, "--dp-emulate is a one-GPU measurement"
    # N > 1: Gaussian-sharded training (the reference's multi-GPU scheme) unless
    # --dp-path asks for the replicated one
    dp_path = args.dp_path
    gshard = world > 1 and not dp_path
    emu_world = args.gshard_emulate
    if emu_world:
        assert world == 1 and not dp_path and emu_world > 1, \
            "--gshard-emulate W: a one-GPU measurement, W > 1"
        gshard = True
    # every eager collective bounded (RCCL's watchdog ends the process on a
    # timeout); captured ones are covered by the progress watchdog below
    import datetime
    pg_kw = {}
    if args.watchdog_s > 0:
        pg_kw["timeout"] = datetime.timedelta(seconds=args.watchdog_s)
    dp_phase = (world > 1 and not dp_path and not args.no_dp_phase) or (
        args.dp_phase and world == 1 and not dp_path and not emu_world and not args.probe)
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), **pg_kw)
    elif args.dp_path or dp_phase:  # a 1-rank RCCL group: the N>1 code path on one GPU
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", local), **pg_kw)
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
    kw = {}
    start = 0
    if args.mcmc:  # simple_trainer.py:1098-1107 (the mcmc preset)
        from gsplat_hip.mcmc import MCMCStrategyConfig
        assert model == "3dgs", "--mcmc: the 3DGS trainer"
        kw = dict(strategy=MCMCStrategyConfig(), sh_degree_interval=1000, max_steps=30_000,
                  init="sfm", init_opacity=0.5, init_scale=0.1, opacity_reg=0.01,
                  scale_reg=0.01)
        start = max(0, REFINE_AT - args.warmup - args.steps // 2)
    elif args.config in DENSIFY:
        from gsplat_hip.densify import DefaultStrategyConfig
        kw = dict(strategy=DefaultStrategyConfig(), sh_degree_interval=1000, max_steps=30_000,
                  init="sfm")
        start = max(0, REFINE_AT - args.warmup - args.steps // 2)
    t_world = emu_world or world
    if emu_world:
        # the peers' rows for rank 0, from their own renders (distributed.Emulation)
        from gsplat_hip import distributed as gdist
        gdist.EMULATION = gdist.Emulation(emu_world)
        for j in range(1, emu_world):
            peer = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device=dev,
                           world_size=emu_world, rank=j, model=model, gaussian_shard=True,
                           graph=False, **kw)
            gdist.EMULATION.record(j, lambda: peer.render(peer.camera_index(start),
                                                          peer.sh_degree_at(start)))
            del peer
        torch.cuda.empty_cache()
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device=dev, world_size=t_world,
                 rank=rank, model=model, sharded_optimizer=dp_path, gaussian_shard=gshard,
                 dp_emulate_world=args.dp_emulate or None,
                 graph=not (args.eager or args.probe
                            or (args.config in DENSIFY and not args.graph and not args.mcmc)),
                 **kw)
    N = means.shape[0]
    # progress watchdog: a rank that stops making progress (a collective a
    # peer never joins, captured or eager) ends the job with its rank, step
    # and phase on stderr and status 3 -- never a silent hang
    from gsplat_hip.distributed import Watchdog
    wd = Watchdog(args.watchdog_s, f"bench.py rank {rank}/{world}") \
        if args.watchdog_s > 0 and not args.probe else None
    hang = tuple(int(x) for x in args.debug_hang.split(":")) if args.debug_hang else None

    def beat(phase, it, trainer):
        if wd is not None:
            g = getattr(trainer, "_graph", None)
            mode = ("eager" if g is None else "capture pending" if g.graph is None
                    else f"replay (captures {g.recaptures}, replays {g.replays})")
            wd.beat(f"rank {rank} {phase} step {it}: {mode}")
        if hang is not None and hang == (rank, it):  # debug: this rank never joins step it
            print(f"bench.py: rank {rank} skips step {it} (--debug-hang)", file=sys.stderr,
                  flush=True)
            time.sleep(1e6)

    if wd is not None:
        wd.arm(f"rank {rank} trainer built")
    for it in range(start, start + args.warmup):
        beat("warmup", it, tr)
        tr.step(it)
    torch.cuda.synchronize()
    if args.probe:  # PMC child run: a few steps, no output
        for it in range(start + args.warmup, start + args.warmup + 2):
            tr.step(it)
        torch.cuda.synchronize()
        return

    timers = _wrapper.enable_kernel_timers(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(start + args.warmup, start + args.warmup + args.steps):
        beat("timed", it, tr)
        tr.step(it)
    beat("timed sync", start + args.warmup + args.steps, tr)
    tr.sync()  # graph replays: every step's overflow check settled inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    # (after the timed region: a failed capture falls back to eager steps)
    graphed = getattr(tr, "_graph", None) is not None
    graph_info = None
    if graphed:
        # kernel durations: a graph replay runs the same kernels as an eager
        # step, but HIP events cannot be recorded per replay -- time the
        # rasterizer launches over eager steps right after the timed region
        graph_info = _graph_info(tr._graph)
        tr.release_graph()  # (RCCL: before destroy_process_group, GraphStep.release)
        timers = _wrapper.enable_kernel_timers(True)
        n_t = min(args.steps, 10)
        for it in range(start + args.warmup + args.steps,
                        start + args.warmup + args.steps + n_t):
            beat("kernel timing", it, tr)
            tr.step(it)
        torch.cuda.synchronize()
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
    # backward (SURVEY §8 d): the forward's gathered record plus an 8-B
    # read-modify-write per gradient field (3DGS: D colour + 2 means2d + 3
    # conic + 1 opacity; 2DGS: D colour + 3 normal + 9 ray transform +
    # 2 means2d + 1 opacity); per pixel the forward outputs it re-reads and
    # the incoming gradients (3DGS: colour 4D + alpha 4 + render alpha 4 +
    # last id 4; 2DGS: the same plus normal 12, distortion 4, median 8).
    per_isect_bwd = per_isect + 8 * ((D + 15) if two else (D + 6))
    per_px_bwd = (4 * D + 40) if two else (4 * D + 12)
    node_name = "_RasterizeToPixels2DGSBackward" if two else "_RasterizeToPixelsBackward"
    last_slot = 12 if two else 9
    byts, byts_bwd, isects, n_effs = [], [], [], []
    for it in range(start + args.warmup, start + args.warmup + min(args.steps, len(vm_pool))):
        beat("roofline bytes", it, tr)
        ci = tr.camera_index(it)
        colors, alphas, meta = tr.render(ci)
        # last_ids are internal to the autograd node (the forward's saved
        # tensors); n_eff = sum over tiles of min(end, max last_id + 1) - start
        offs = meta["isect_offsets"].flatten().long()
        n = meta["flatten_ids"].numel()
        ends = torch.cat([offs[1:], torch.tensor([n], device=dev)])
        node = colors.grad_fn
        while node is not None and type(node).__name__ != node_name:
            node = node.next_functions[0][0]
        last = node.saved_tensors[last_slot] if node is not None else None
        ts = meta["tile_size"]
        tw, th = meta["tile_width"], meta["tile_height"]
        if last is not None:
            lp = torch.nn.functional.pad(last[0], (0, tw * ts - W, 0, th * ts - H))
            tmax = lp.view(th, ts, tw, ts).amax(dim=(1, 3)).flatten().long()
            n_eff = int(torch.clamp(torch.minimum(ends, tmax + 1) - offs, min=0).sum())
        else:
            n_eff = n
        P = H * W
        byts.append(n_eff * per_isect + P * per_px + 4 * tw * th)
        byts_bwd.append(n_eff * per_isect_bwd + P * per_px_bwd + 4 * tw * th)
        isects.append(n)
        n_effs.append(n_eff)
        del colors, alphas, meta, node, last
    # fraction of the Gaussians visible from at least one of the pool's first
    # 8 cameras -- what a replicated 8-GPU step would have to reduce
    # (DESIGN §6); projection only, outside the timed region
    union_visible = per_cam_visible = None
    if model == "3dgs":
        from gsplat_hip import fully_fused_projection
        p = tr.params
        nc = min(8, len(vm_pool))
        with torch.no_grad():
            radii = fully_fused_projection(
                p["means"], None, p["quats"], torch.exp(p["scales"]), tr.viewmats[:nc],
                tr.Ks[:nc], W, H, packed=False, near_plane=0.01, far_plane=1e10)[0]
        union_visible = float((radii > 0).any(0).float().mean())
        per_cam_visible = float((radii > 0).float().mean())
    bytes_per_launch = float(np.mean(byts))
    bytes_bwd = float(np.mean(byts_bwd))
    achieved = bytes_per_launch / (fwd_ms * 1e-3) / 1e9
    achieved_bwd = bytes_bwd / (bwd_ms * 1e-3) / 1e9

    pf = None if traffic is None else traffic["fwd"]
    pb = None if traffic is None else traffic["bwd"]
    result = {
        "metric": "train-step images/sec + rasterize fwd HBM GB/s, garden 1080p, 1/2/4/8 MI355X",
        "value": world * args.steps / elapsed,
        "unit": "images/s",
        "n_gpus": dist.get_world_size() if world > 1 else 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: garden SfM points (assets/test_garden.npz crop) tiled "
                f"{grid}x{grid}, random scales/quats/opacities, random target images",
        "config": {"workload": desc, "gaussians": N,
                   "gaussians_after": int(sum(tr._n_world) if gshard
                                          else tr.params["means"].shape[0]),
                   "first_timed_step": start + args.warmup, "width": W, "height": H,
                   "cameras_per_rank_per_step": 1,
                   "parallelism": (
                       f"gshard{emu_world} emulated on one GPU: the per-rank step of rank 0 "
                       f"(Gaussians [0::{emu_world}], its own camera, projection + SH into "
                       f"{emu_world} cameras, rasterization with all Gaussians, per-shard Adam); "
                       "the other ranks' exchanged rows are stand-ins recorded from their own "
                       "renders and the exchanges are device copies of the same rows -- no "
                       "xGMI time (measurement only)") if emu_world else (
                       f"gshard{world}: rank r holds Gaussians [r::{world}] and renders its own "
                       "camera; projected pairs exchanged peer to peer over RCCL/xGMI "
                       "(rasterization(distributed=True)), per-shard Adam, no gradient "
                       "all-reduce") if gshard else f"dp{world}" + (
                       f" emulating the per-rank compute of dp{args.dp_emulate}: optimizer rows "
                       f"sharded {args.dp_emulate} ways, this rank's share updated, no "
                       "collectives executed (measurement only)" if args.dp_emulate else
                       " (the N>1 code path on a 1-rank RCCL group: sharded Adam, "
                       "early SH reduce-scatter)" if dp_path and world == 1 else ""),
                   # bytes this rank sends to its peers per step (distributed.exchange_pairs:
                   # 48 B per (Gaussian, peer camera) forward, 40 B of gradients back)
                   "exchange_bytes_out_per_rank": (
                       {"forward": 48 * tr.params["means"].shape[0] * (len(tr._n_world) - 1),
                        "backward": 40 * tr.params["means"].shape[0] * (len(tr._n_world) - 1)}
                       if gshard else None),
                   "n_isects_mean": float(np.mean(isects)), "n_eff_mean": float(np.mean(n_effs)),
                   "fwd_split_div": getattr(tr, "split_div", None),
                   "termination_ratio_first_render": getattr(tr, "term_ratio", None),
                   "visible_per_camera": per_cam_visible,
                   "visible_union_8_cameras": union_visible,
                   "packed": False, "loss": "0.8*L1+0.2*(1-SSIM valid)",
                   "step_issue": ("HIP graph replay of the captured step (sync-free isect, "
                                  f"{graph_info})" if graphed else "eager launches" + (
                                      f" (graph capture failed: {tr.graph_fallback})"
                                      if getattr(tr, "graph_fallback", None) else "")),
                   "optimizer": "Adam (6 groups)" + (
                       ", each rank on its own Gaussians" if gshard else
                       ", sharded over ranks" if dp_path else
                       ", SH groups' step fused into the SH backward"
                       if getattr(tr, "sh_adam_in_bwd", False) else ""),
                   "densification": tr.densify_desc()},
        "roofline": {"kernel": kname, "bound": "hbm", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None if pf is None else pf["bytes_per_launch"],
                     "traffic_detail": pf,
                     "algorithmic_bytes_per_launch": bytes_per_launch,
                     "bytes_per_isect": per_isect, "bytes_per_pixel": per_px,
                     "launch_ms": fwd_ms,
                     "launch_ms_source": ("HIP events around the launch on its stream, over "
                                          + ("eager steps right after the graph-replayed timed "
                                             "region (same kernels)" if graphed else
                                             "the timed region")),
                     # the kernel's binding ceiling is VALU issue, not HBM
                     "valu": _valu_frac(pf, fwd_ms),
                     "bwd": {"kernel": kname.replace("fwd", "bwd"), "bound": "hbm",
                             "achieved": achieved_bwd, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": achieved_bwd / HBM_PEAK_GBS,
                             "traffic": None if pb is None else pb["bytes_per_launch"],
                             "traffic_detail": pb,
                             "algorithmic_bytes_per_launch": bytes_bwd,
                             "bytes_per_isect": per_isect_bwd, "bytes_per_pixel": per_px_bwd,
                             "launch_ms": bwd_ms, "valu": _valu_frac(pb, bwd_ms)},
                     "pmc_source": None if traffic is None else traffic["source"],
                     "pmc_note": None if world == 1 else "PMC passes run at N=1 only "
                                 "(per-GPU workload is the same at every N)"},
        "model": model,
    }
    if dp_path:  # the main region IS the replicated data-parallel scheme
        result["config"]["dp"] = {"phase": "main", "value": result["value"],
                                  "ms_per_step": result["ms_per_step"],
                                  "step_issue": result["config"]["step_issue"]}
    if rank == 0 and not args.no_cpu_baseline:
        # after the timed region; the other ranks wait at the barrier below
        if wd is not None:
            wd.disarm()  # host-only work of bounded length (tens of seconds)
        try:
            result["cpu_baseline"] = cpu_baseline(tr, args.cpu_tile_stride, cpu_pool)
        finally:
            cpu_pool.close()
        if wd is not None:
            wd.arm(f"rank {rank} cpu baseline done")
    if dp_phase:
        # north_star's own multi-GPU scheme, timed in the same job after the
        # main (Gaussian-sharded) region: replicated Gaussians, per-camera
        # data parallelism, gradients reduce-scattered and rows all-gathered
        # over RCCL (distributed.ShardedAdam).  A failure is recorded here
        # without losing the main value; a hang ends the job through the
        # watchdog, which then still delivers the main line (dp: "hung")
        if wd is not None:
            hung = dict(result, config=dict(result["config"], dp={
                "error": f"hung: no progress for {args.watchdog_s:.0f} s (watchdog)"}))
            wd.fallback(json_fd if rank == 0 else 2,
                        json.dumps(hung) + "\n" if rank == 0 else "", 0)
        tr.release_graph()
        del tr
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        try:
            result["config"]["dp"] = dp_region(args, means, rgbs, vm_pool, K_pool, W, H, dev, world,
                                               rank, start, kw, beat)
        except Exception as e:  # noqa: BLE001 -- recorded, the main value stands
            import traceback
            traceback.print_exc()
            result["config"]["dp"] = {"error": repr(e)[:400]}
        if wd is not None:
            wd.fallback(-1, None)
        tr = None
    if rank == 0:
        os.write(json_fd, (json.dumps(result) + "\n").encode())
    if world > 1:
        dist.barrier()
    if wd is not None:
        wd.disarm()
    if dist.is_initialized():
        if tr is not None:
            tr.release_graph()
        import gc
        gc.collect()  # graphs that captured RCCL collectives, before the group goes
        torch.cuda.synchronize()
        dist.destroy_process_group()


def _graph_info(g):
    return {"replays": g.replays, "captures": g.recaptures,
            "capture_ms": [round(1e3 * x, 1) for x in g.capture_s],
            "isect_capacity": g.capacity, "max_isects": g.max_isects,
            "host_issue_ms_per_step": 1e3 * g.host_s / max(g.replays, 1)}


def dp_region(args, means, rgbs, vm_pool, K_pool, W, H, dev, world, rank, start, kw, beat):
    """The replicated per-camera data-parallel step (Trainer(sharded_optimizer=
    True), graph-replayed with its RCCL collectives inside), timed like the
    main region: barrier + synchronize on both sides, max over ranks."""
    from gsplat_hip.train_step import Trainer
    if world == 1:
        os.environ["GSPLAT_HIP_DP_SOLO"] = "0"  # the collectives on the 1-rank group
    tr = Trainer(means, rgbs, vm_pool, K_pool, W, H, sh_degree=3, device=dev, world_size=world,
                 rank=rank, sharded_optimizer=True, gaussian_shard=False,
                 graph=not args.eager, **kw)
    try:
        for it in range(start, start + args.warmup):
            beat("dp warmup", it, tr)
            tr.step(it)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(start + args.warmup, start + args.warmup + args.steps):
            beat("dp timed", it, tr)
            tr.step(it)
        beat("dp timed sync", start + args.warmup + args.steps, tr)
        tr.sync()
        torch.cuda.synchronize()
        dist.barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
        g = getattr(tr, "_graph", None)
        issue = (f"HIP graph replay with the RCCL reduce-scatters / all-gathers inside "
                 f"({_graph_info(g)})" if g is not None else "eager launches" + (
                     f" (graph capture failed: {tr.graph_fallback})" if tr.graph_fallback else ""))
        return {"phase": "second timed region (after the main one)", "value": world * args.steps / elapsed,
                "unit": "images/s", "ms_per_step": 1e3 * elapsed / args.steps,
                "steps": args.steps, "warmup": args.warmup, "step_issue": issue,
                "parallelism": f"dp{world}: every rank holds all Gaussians and renders its own "
                               "camera; gradients reduce-scattered, Adam on the rank's rows, rows "
                               "all-gathered over RCCL (sharded optimizer)"}
    finally:
        tr.release_graph()


def host_threads() -> int:
    """Host cores this job may use: the box's share (OMP_NUM_THREADS, set to
    the GPU's CPU share on the GPU box) or, failing that, the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env)) if env and env.isdigit() else aff)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(tr, stride, pool):
    """The numpy oracle's train step (oracle/cpu_step.py) on the host's cores."""
    from oracle.cpu_step import cpu_train_step
    p = {k: v.detach().cpu().numpy() for k, v in tr.params.items()}
    sh = np.concatenate([p["sh0"], p["shN"]], 1)
    ci = 0
    threads = pool.workers
    if stride <= 0:  # auto: whole image with >= 8 threads, else a 1/24 tile sample
        stride = 1 if threads >= 8 else 24
    total, parts, sample = cpu_train_step(
        p["means"], p["quats"], p["scales"], p["opacities"], sh, tr.viewmats[ci].cpu().numpy(),
        tr.Ks[ci].cpu().numpy(), tr.width, tr.height, tr.targets[ci].cpu().numpy(),
        tile_stride=stride, pool=pool)
    return {"value": 1.0 / total, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": sample, "seconds_per_step": total,
            "breakdown_s": {k: round(v, 3) for k, v in parts.items()},
            "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}


if __name__ == "__main__":
    main()
