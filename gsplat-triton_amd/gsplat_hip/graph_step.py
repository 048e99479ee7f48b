"""The training step captured into a HIP graph and replayed.

Eager, a step is ~70 host-side launches plus the one host synchronisation of
the tile intersection (the reference's `.item()` of n_isects,
gsplat/triton_impl/isect_tiles.py:101-102).  On a slow host the GPU waits
for the launches (one box ran 520 against 731 images/s with
identical kernel times).  Here the step is captured once with
torch.cuda.CUDAGraph (HIP graphs on ROCm) and replayed: one replay, two
small host->device copies and one device->host copy per step.

What makes the step capturable:
* the sync-free intersection (`rasterization(_isect_capacity=...)`,
  gsplat_hip_isect_write_sorted_capped): isect arrays of a fixed capacity,
  every count stays on the device;
* the step-dependent inputs -- the Adam factors lr / (1 - b1^t),
  1 / sqrt(1 - b2^t) with the means learning-rate schedule
  (gsplat_hip_adam_step_dev, gsplat_hip_sh_colors_bwd_adam_dev; computed with
  the eager path's own arithmetic, losses.adam_factors), the camera's
  viewmat and K, and its index (the loss reads that camera's target image
  in place, l1_ssim_loss(gt_index=...)) -- are one 512-B block.  The host
  writes it into a slot of a host-mapped ring; the graph's first kernel
  (the activations, gsplat_hip_activate_fwd_fetch) copies slot seq % RING
  into device memory and counts seq up, so a step needs no copy-engine
  transfer (each one cost a
  cross-queue hand-off of ~15 us before and after it);
* overflow: if a step's isects do not fit, the capped emission writes none,
  sets a sticky device flag, and every state update of that and the later
  steps reads the flag and does nothing.  The emission also writes each
  step's counts into that step's row of a host-mapped ring; the host reads
  them once the step is done (up to `lag` steps late), then waits for the
  GPU, grows the capacity, re-captures and re-runs the void steps in order
  -- so the result is the eager step sequence's.

Scope: the fused 3DGS trainer -- one rank (the bench's M2 and, with its
DefaultStrategy schedule, M3 configurations; with MCMCStrategy the position
noise is a launch of the captured step, its step index and scale in the
input block), Gaussian-sharded (its pair
exchanges inside the graph) and per-camera data parallel with the sharded
optimizer (its reduce-scatters, Adam and all-gathers inside the graph): the
steps between two refines are replays of one capture; a refine (eager,
after its step's replay has been checked) replaces the parameter tensors,
and the next step re-captures with an isect capacity grown in proportion to
the Gaussians.  Anything else runs eagerly (Trainer.step).

Several ranks: a rank whose isects overflow voids its step, and its
gradients reach the other ranks' updates (the exchanges, the reductions),
so the ranks agree on the flag inside the graph (a MAX all-reduce of it,
issued after the forward and waited for before the backward, beside the
loss kernels) and write the agreed flag into their count rings
(gsplat_hip_status_to_ring); each rank checks its steps in issue order at
fixed points (no opportunistic early check), so all ranks recover from the
same step and re-capture together.
"""

import collections
import ctypes
import gc
import math
import os
import time

import numpy as np
import torch

from . import _lib, _wrapper
from .losses import FusedAdam, adam_factors, l1_ssim_loss
from .rendering import rasterization, rasterization_2dgs
from . import mcmc as _mcmc
from .strategy import activate, update_state_


class GraphCaptureError(RuntimeError):
    """A capture of the training step failed (on this rank or, for a
    Gaussian-sharded job, on any rank: the ranks agree before replaying).
    Trainer.step catches it and runs the steps eagerly from then on, in the
    same process."""


def graphable(tr) -> bool:
    """Whether Trainer `tr` can run its steps as graph replays.  With a
    DefaultStrategy or MCMCStrategy schedule the steps between refines are
    replays (MCMC's position noise inside them); the refine / opacity reset
    run eagerly after their step (Trainer.step), and a refine (new parameter
    tensors, Trainer._param_gen) re-captures."""
    st = tr.strategy
    # Gaussian-sharded (one camera per rank): its two pair exchanges inside
    # the graph -- RCCL's all_to_all_single (the default at N > 1; the
    # capture is checked on a one-rank RCCL group by
    # tests/test_gpu_distributed.py; GSPLAT_HIP_GRAPH_RCCL=0 issues those
    # steps eagerly) or the device copies of the one-GPU emulation
    # (distributed.EMULATION, bench --gshard-emulate)
    from . import distributed as gdist
    rccl_ok = os.environ.get("GSPLAT_HIP_GRAPH_RCCL", "1") != "0"
    gshard_ok = (getattr(tr, "gshard", False) and tr.world_size <= GraphStep.MAX_WORLD
                 and isinstance(tr.opt, FusedAdam) and (gdist.EMULATION is not None or rccl_ok))
    # per-camera data parallelism with the sharded optimizer (bench --dp-path):
    # its reduce-scatters / all-gathers inside the graph (none on a one-rank
    # group, distributed.ShardedAdam.solo)
    dp_ok = (tr.sharded and isinstance(tr.opt, gdist.ShardedAdam)
             and (tr.opt.solo or rccl_ok))
    one = tr.world_size == 1 and not getattr(tr, "gshard", False) and not tr.sharded
    # one rank: 3DGS or 2DGS (surfels, rasterization_2dgs with the sync-free isect)
    return (tr.fused and (tr.model == "3dgs" or (one and tr.model == "2dgs"))
            and (gshard_ok or dp_ok or (one and isinstance(tr.opt, FusedAdam)))
            and not getattr(tr, "packed", False)
            and (st is None or (not getattr(st, "absgrad", False) and tr.radii2d is None))
            and torch.device(tr.device).type == "cuda")


NODE_TYPES = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event",
              "event_record")


def graph_node_census(g):
    """{node type: count} of a captured torch.cuda.CUDAGraph(keep_graph=True),
    and the memset nodes as (address, bytes per row, rows, element size)."""
    counts = (ctypes.c_int64 * 16)()
    ms = (ctypes.c_int64 * (4 * 64))()
    _lib.call("gsplat_hip_graph_node_census", ctypes.c_void_p(g.raw_cuda_graph()),
              ctypes.addressof(counts), ctypes.addressof(ms), 64)
    names = {(NODE_TYPES[t] if t < len(NODE_TYPES) else f"type{t}"): int(c)
             for t, c in enumerate(counts) if c}
    n_ms = min(names.get("memset", 0), 64)
    return names, [tuple(int(x) for x in ms[4 * k:4 * k + 4]) for k in range(n_ms)]


def graph_memcpy_census(g):
    """(destination, source, bytes, hipMemcpyKind) of every memcpy node of a
    captured graph (-1 where unreadable)."""
    out = (ctypes.c_int64 * (4 * 64))()
    n = ctypes.c_int(0)
    _lib.call("gsplat_hip_graph_memcpy_census", ctypes.c_void_p(g.raw_cuda_graph()),
              ctypes.addressof(out), 64, ctypes.addressof(n))
    return [tuple(int(x) for x in out[4 * k:4 * k + 4]) for k in range(min(n.value, 64))]


def check_kernel_nodes_only(g, allow_d2d=False):
    """The captured step must hold kernel (and empty) nodes only: its replays
    faulted with the backward's hipMemsetAsync nodes in the graph (DESIGN
    §3.12), so a memset / copy that slips into the captured region (a
    torch.zeros, a .copy_) fails here, at capture time.  `allow_d2d`: the
    Gaussian-sharded step's RCCL exchanges may add memcpy nodes (RCCL
    copies a one-rank group's own block with them); memset nodes still fail."""
    names, memsets = graph_node_census(g)
    allowed = ("kernel", "empty")
    if names.get("memcpy"):
        cps = graph_memcpy_census(g)
        # RCCL's copies: torch's bundled HIP runtime returns garbage from
        # hipGraphMemcpyNodeGetParams for the 1-D memcpy nodes a captured
        # hipMemcpyAsync makes (profiles/r5/rccl_capture.txt), so their kind
        # cannot be checked here; their replay is checked against eager steps
        # by tests/test_gpu_distributed.py (one-rank RCCL group)
        if allow_d2d:
            allowed = allowed + ("memcpy",)
        names = dict(names, memcpy_nodes=[(hex(d), hex(s_), b, k) for d, s_, b, k in cps])
    other = {k: v for k, v in names.items() if k not in allowed and k != "memcpy_nodes"}
    if "memcpy" in other:
        other["memcpy_nodes"] = names["memcpy_nodes"]
    if other:
        raise RuntimeError(f"captured training step holds non-kernel nodes {other}; memset "
                           f"nodes (address, row bytes, rows, element size): {memsets}")
    return names


class _Mapped:
    """Host-mapped, coherent memory (gsplat_hip_host_mapped_alloc): `np` for
    the host, `dev` (a pointer) for kernels.  Never freed: a captured graph
    keeps the device pointer in its kernel arguments and may still be
    replaying when its GraphStep becomes garbage, and freeing pinned memory
    from a garbage-collector pass aborted a test process; the rings are
    4.3 KB per GraphStep."""

    def __init__(self, nbytes):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("gsplat_hip_host_mapped_alloc", int(nbytes), ctypes.addressof(h),
                  ctypes.addressof(d))
        self.host, self.dev = h.value, d.value
        self.np = np.ctypeslib.as_array((ctypes.c_uint8 * int(nbytes)).from_address(self.host))


class GraphStep:
    """Trainer.step as HIP graph replays (see the module docstring)."""

    RING = 8  # host-mapped slots for the per-step input block and counts
    SLOT = 2048  # bytes per input block
    LOSS_RING = 4096  # device slots of the returned per-step losses
    MAX_WORLD = 8  # cameras of a Gaussian-sharded step in the block

    def __init__(self, tr, capacity=None, headroom=1.25, lag=2):
        assert graphable(tr), "GraphStep: a fused 3DGS trainer (graph_step.graphable)"
        self.tr = tr
        dev = torch.device(tr.device)
        self.dev = dev
        self.headroom = float(headroom)
        self.lag = int(lag)  # steps the host may run ahead of its overflow check
        self.capacity = None if capacity is None else int(capacity)
        # device input of the graph: one 2-KB block per step -- f32 [0, 64)
        # the Adam factors, i64 at byte 256 the rank's camera index, f32
        # viewmats [W][16] at byte 512 and Ks [W][9] at
        # byte 1024 (W = the world's cameras: 1, or the Gaussian-sharded job's
        # ranks), the camera-to-world matrix f32 [16] at byte 1536 (2DGS: its
        # normals), MCMC's step i64 / noise scale f32 at bytes 264 / 272,
        # i64 at SLOT - 8 the ring slot (written by
        # gsplat_hip_step_fetch)
        self.n_groups = len(tr.params)
        self.gshard = bool(getattr(tr, "gshard", False))
        self.dp = bool(tr.sharded)  # per-camera data parallel, distributed.ShardedAdam
        self.W = tr.world_size if self.gshard else 1
        # the ranks agree on the overflow flag inside the graph (module docstring)
        import torch.distributed as dist
        from . import distributed as gdist
        self.vote = ((self.gshard or self.dp) and gdist.EMULATION is None
                     and dist.is_available() and dist.is_initialized())
        # the captured collectives' own communicator: never any eager work on
        # it (distributed._CAPTURE_PG); None where the step has no collective
        # (a one-rank data-parallel step with the collectives skipped still
        # votes, on a one-rank group)
        self.cap_pg = None
        if self.vote and dist.get_backend() == "nccl":
            self.cap_pg = gdist.new_capture_group()
        self.blk = torch.zeros(self.SLOT, dtype=torch.uint8, device=dev)
        self.scal = self.blk[:256].view(torch.float32)
        self.cam = self.blk[256:264].view(torch.int64)
        self.vm_w = self.blk[512:512 + 64 * self.W].view(torch.float32).view(self.W, 4, 4)
        self.K_w = self.blk[1024:1024 + 36 * self.W].view(torch.float32).view(self.W, 3, 3)
        r = tr.rank if self.gshard else 0
        self.vm, self.K = self.vm_w[r:r + 1], self.K_w[r:r + 1]  # this rank's camera
        self.c2w = self.blk[1536:1536 + 64].view(torch.float32).view(1, 4, 4)
        # MCMC: the step index (i64 at byte 264) and its noise scale (f32 at 272)
        self.mstep = self.blk[264:272].view(torch.int64)
        self.mscale = self.blk[272:276].view(torch.float32)
        self.slot = self.blk[self.SLOT - 8:].view(torch.int64)
        self.seq = torch.zeros(1, dtype=torch.int64, device=dev)  # steps fetched
        # the step's loss, written by the loss's own reduction launch into
        # slot (seq - 1) % LOSS_RING: step() returns that slot, no copy launch
        # after the replay (a 4-B device copy cost ~4 us of GPU time a step);
        # a returned loss stays valid for LOSS_RING later steps
        self.loss_ring = torch.zeros(self.LOSS_RING, dtype=torch.float32, device=dev)
        self.ring_loss = not (getattr(tr, "opacity_reg", 0.0) > 0.0 or
                              getattr(tr, "scale_reg", 0.0) > 0.0)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)  # sticky overflow flag
        self.ring_in = _Mapped(self.RING * self.SLOT)
        self.ring_out = _Mapped(self.RING * 4 * 8)
        self._out = self.ring_out.np.view(np.int64).reshape(self.RING, 4)
        self._slot_ev = [None] * self.RING
        self._vm_host = tr.viewmats.detach().float().cpu().numpy()
        self._K_host = tr.Ks.detach().float().cpu().numpy()
        self.graph = None
        self.key = None
        self.counts = None  # the graph's isect counts (device i64[4])
        self.loss = None
        # (it, slot, event, seq, returned loss) awaiting the overflow check
        self.pending = collections.deque()
        self.issued = 0
        self.recaptures = 0
        self.capture_s = []  # host seconds per capture (warm-up, capture, instantiate)
        self.replays = 0
        self.max_isects = 0
        self.host_s = 0.0
        # set when a recovery's re-capture failed (its voided steps were then
        # re-run eagerly): Trainer.step issues every later step eagerly
        self.failed = None

    # ------------------------------------------------------------------ body
    def _layout(self):
        """(groups of the Adam launches in launch order, offset of the SH-Adam
        factors): the device-side factors are laid out in that order."""
        if self.dp:
            idx = [i for sel in self.tr.opt.launch_plan() for i in sel]
            return idx, 2 * len(idx)
        names = list(self.tr.params)
        sh = {names.index("sh0"), names.index("shN")}
        idx = [i for i in range(self.n_groups) if not (self.tr.sh_adam_in_bwd and i in sh)]
        return idx, 2 * len(idx)

    def _body(self, deg, stats=True):
        tr = self.tr
        p = tr.params
        names = list(p)
        idx, sh_off = self._layout()
        fa = None
        if tr.sh_adam_in_bwd:
            o = tr.opt
            i0, i1 = names.index("sh0"), names.index("shN")
            fa = _wrapper.ShAdamInBackward(
                p["sh0"].data, p["shN"].data, o.exp_avg[i0], o.exp_avg_sq[i0], o.exp_avg[i1],
                o.exp_avg_sq[i1], o.lrs[i0], o.lrs[i1], o.betas, o.eps, 1,
                hyper=self.scal[sh_off:sh_off + 3], skip=self.status)
        ga = None
        if getattr(tr, "geom_in_proj", False):
            # the geometry groups' factors are the first launch groups' (_fill):
            # (ss, ib) of means, scales, quats, opacities at [0, 8); the SH
            # groups follow when their update is not fused into the SH backward
            assert [names[i] for i in idx][:len(tr.GEOM)] == list(tr.GEOM), (idx, names)
            ga = tr.geom_adam_in_backward(1, hyper=self.scal[:2 * len(idx)], skip=self.status)
        fusion = _wrapper.StepFusion(sh_adam=fa, geom=tr.geom_fuse, geom_adam=ga) \
            if (fa is not None or tr.geom_fuse) else None
        # the first launch also fetches this step's input block (the ring slot)
        scales, opac = activate(p["scales"], p["opacities"], fusion,
                                fetch=(self.ring_in.dev, self.SLOT, self.RING, self.seq, self.blk))
        dkw = {}
        if self.gshard:  # the world's cameras from the block, shard sizes fixed per capture
            dkw = dict(distributed=True, _world_cameras=(self.vm_w, self.K_w),
                       _world_counts=tr._n_world)
        grad_box = {}
        if tr.model == "2dgs":  # Trainer.render's call, with the sync-free isect
            rc, _, _, _, _, _, meta = rasterization_2dgs(
                p["means"], p["quats"], scales, opac, (p["sh0"], p["shN"]), self.vm, self.K,
                tr.width, tr.height, sh_degree=deg, packed=False, near_plane=0.01,
                far_plane=1e10, render_mode="RGB+D", _fusion=fusion,
                _isect_capacity=self.capacity, _isect_status=self.status,
                _isect_report=(self.ring_out.dev, self.slot), _camtoworlds=self.c2w,
                _colors_only=True)
            colors = rc  # the loss reads the colour channels in place (_channels=3)
            # the densification input is a leaf: its .grad after the backward
            # (a hook keeping a reference would make AccumulateGrad clone the
            # gradient -- a memcpy node in the graph)
        else:
            with _wrapper.fwd_split(getattr(tr, "split_div", None),
                                    getattr(tr, "split_threshold", None)):
                colors, _, meta = rasterization(
                    p["means"], p["quats"], scales, opac, (p["sh0"], p["shN"]), self.vm, self.K,
                    tr.width, tr.height, sh_degree=deg, packed=False, near_plane=0.01,
                    far_plane=1e10, radius_clip=0.0,
                    rasterize_mode=getattr(tr, "rasterize_mode", "classic"), _fusion=fusion,
                    _isect_capacity=self.capacity, _isect_status=self.status,
                    _isect_report=(self.ring_out.dev, self.slot), _isect_ids=False, **dkw)
            meta["means2d"].register_hook(lambda g: grad_box.__setitem__("g", g))
        vote = None
        if self.vote:  # the ranks' overflow flags, agreed beside the loss kernels
            import torch.distributed as dist
            from . import distributed as gdist
            vote = dist.all_reduce(self.status, op=dist.ReduceOp.MAX, async_op=True,
                                   group=gdist.current_capture_group())
        loss = tr._regularise(l1_ssim_loss(
            colors, tr.targets, tr.ssim_lambda, gt_index=self.cam,
            _out_ring=(self.loss_ring, self.seq) if self.ring_loss else None,
            _channels=3 if tr.model == "2dgs" else None))
        if vote is not None:
            vote.wait()
            _lib.call("gsplat_hip_status_to_ring", self.status.data_ptr(), self.ring_out.dev,
                      self.slot.data_ptr(), _wrapper._stream())
        from . import losses as _losses
        tr._sh_ready = 0  # the sharded optimizer's SH reduce-scatter hook
        if self.dp:  # its collectives in order on this stream (ShardedAdam.capturing)
            tr.opt.capturing = True
        try:
            torch.autograd.backward(loss, _losses.ONE_GRAD)
            if tr.model == "2dgs" and meta["gradient_2dgs"].grad is not None:
                grad_box["g"] = meta["gradient_2dgs"].grad
            if stats and "g" in grad_box:  # DefaultStrategy statistics (until refine_stop_iter)
                update_state_(tr.grad2d, tr.count, grad_box["g"], meta["radii"], meta["width"],
                              meta["height"], meta["n_cameras"], skip=self.status)
            if self.dp:  # reduce-scatter, Adam on this rank's rows, all-gather: all inside
                assert not tr._sh_skip(fusion)
                tr.opt.step(defer_gather=False, xform=tr._geom_xform(fusion),
                            hyper=self.scal[:sh_off], void=self.status)
            else:
                skip = tr._sh_skip(fusion)
                launched = tuple(i for i in range(self.n_groups) if i not in skip)
                # the launched groups are the launch plan's tail (the geometry
                # groups, its head, may have been updated by the projection
                # backward): their factors start at that offset
                assert launched == tuple(idx[len(idx) - len(launched):]), (skip, idx)
                off = 2 * (len(idx) - len(launched))
                tr.opt.step(skip=skip, xform=tr._geom_xform(fusion),
                            hyper=self.scal[off:sh_off], void=self.status)
        finally:
            # (also when the body raises: later eager steps use the optimizer's
            # own streams and communicators again)
            if self.dp:
                tr.opt.capturing = False
        tr.opt.zero_grad(set_to_none=True)
        if getattr(tr, "mcmc", False):
            # MCMCStrategy's position noise after the update (Trainer.mcmc_noise):
            # the step and its scale from the block (scale 0 on refine steps,
            # whose noise follows the eager refine), nothing on a void step
            _mcmc.inject_noise({k: p[k].data for k in ("means", "quats", "scales", "opacities")},
                               0.0, seed=tr._noise_seed, step_dev=self.mstep,
                               scaler_dev=self.mscale, skip=self.status)
        return loss, meta["isect_counts"]

    def _capture(self, deg, stats=True):
        t0 = time.perf_counter()
        err = None
        try:
            self._capture_impl(deg, stats)
        except RuntimeError as e:  # a HIP / RCCL / torch failure of the capture:
            # eager fallback (programming errors -- assertions, type errors --
            # propagate)
            err = e
            self.graph, self.key = None, None
        finally:
            self.capture_s.append(time.perf_counter() - t0)
        ok = self._agree(err is None)
        if err is not None:
            raise GraphCaptureError(f"capture failed on this rank: {err!r}") from err
        if not ok:
            self.graph, self.key = None, None
            raise GraphCaptureError("capture failed on another rank")

    def _agree(self, ok: bool) -> bool:
        """A Gaussian-sharded job replays only if every rank captured: one
        MIN all-reduce of the ranks' outcomes, outside the capture (the
        ranks' replays hold matching RCCL exchanges, so all replay or none)."""
        import torch.distributed as dist
        from . import distributed as gdist
        if not (self.vote and self.tr.world_size > 1 and gdist.EMULATION is None
                and dist.is_initialized()):
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(int(t.item()))

    def _capture_impl(self, deg, stats=True):
        tr = self.tr
        from . import losses as _losses
        if _losses.ONE_GRAD is None or _losses.ONE_GRAD.device != self.dev:
            _losses.ONE_GRAD = torch.ones((), device=self.dev)
        if self.capacity is None:
            self.capacity = self._probe_capacity(deg)
        timers = _wrapper._timers
        _wrapper._timers = None  # no timing events inside the graph
        if self.dp:
            tr.opt.wait()  # an eager step's deferred all-gathers
        torch.cuda.synchronize(self.dev)
        try:
            # warm-up on a side stream (torch's capture recipe) as a VOID
            # step: the flag makes every state update a no-op.  Only before
            # the first capture: a re-capture (a refine's new tensors, the SH
            # degree) runs code that has run before, and the warm-up would
            # cost a whole extra step per refine
            self.status.fill_(1)
            if self.recaptures == 0:
                s = torch.cuda.Stream(device=self.dev)
                s.wait_stream(torch.cuda.current_stream(self.dev))
                with torch.cuda.stream(s):
                    self._body(deg, stats)
                torch.cuda.current_stream(self.dev).wait_stream(s)
            self.graph = None
            g = torch.cuda.CUDAGraph(keep_graph=True)
            dump = os.environ.get("GSPLAT_HIP_GRAPH_DUMP")  # diagnosis: the graph as DOT
            if dump:
                g.enable_debug_mode()
            # no garbage collection while capturing: a collected object that
            # owns a HIP resource (an earlier trainer's graph or event) would
            # free it with a call that is illegal during a capture -- a test
            # process aborted there.  torch.cuda.graph collects right before.
            gc_on = gc.isenabled()
            gc.disable()
            # RCCL's watchdog threads query the end events of the eager
            # collectives they track; a query of an event recorded on a stream
            # the capture has pulled in aborted a test process (round 5).  The
            # captured collectives therefore run on a communicator of their
            # own that never issues eager work (self.cap_pg,
            # distributed._CAPTURE_PG; torch does not track collectives issued
            # during a capture), so every event the watchdogs query lives on a
            # stream outside the capture -- by construction, not by timing --
            # and thread-local capture mode keeps their queries legal.
            from . import distributed as gdist
            try:
                with gdist.capture_group(self.cap_pg), \
                        torch.cuda.graph(g, capture_error_mode="thread_local"):
                    self.loss, self.counts = self._body(deg, stats)
            finally:
                if gc_on:
                    gc.enable()
            if dump:
                g.debug_dump(f"{dump}.{self.recaptures}.dot")
            # RCCL's collectives (a Gaussian-sharded or data-parallel step on
            # a real process group) may hold device-to-device copies
            self.census = check_kernel_nodes_only(g, allow_d2d=self.vote)
            g.instantiate()
            self.graph = g
            self.status.zero_()
            self.seq.fill_(self.issued)  # the next replay fetches slot issued % RING
            torch.cuda.synchronize(self.dev)
        finally:
            _wrapper._timers = timers
        self.key = self._key_of(deg, stats)
        self.recaptures += 1

    def _probe_capacity(self, deg):
        """n_isects of the first camera, from one eager render (no grad)."""
        tr = self.tr
        with torch.no_grad():
            _, _, meta = tr.render(0, deg)
            n = int(meta["flatten_ids"].numel())
        return max(1 << 16, int(math.ceil(n * self.headroom)))

    # ------------------------------------------------------------ host side
    def _fill(self, it, slot):
        """The step block of step `it` into pinned slot `slot`."""
        tr = self.tr
        o = tr.opt
        step = o.step_count + 1
        lrs = list(o.lrs)
        if tr.max_steps:  # means ExponentialLR (Trainer.step sets it before Adam)
            lrs[0] = tr.lrs[0] * (0.01 ** (1.0 / tr.max_steps)) ** it
        idx, sh_off = self._layout()
        b = self.ring_in.np[slot * self.SLOT:(slot + 1) * self.SLOT]
        f = b[:256].view(np.float32)
        fac = adam_factors([lrs[i] for i in idx], o.betas, step)
        for k, (ss, ib) in enumerate(fac):
            f[2 * k], f[2 * k + 1] = ss, ib
        if tr.sh_adam_in_bwd:
            names = list(tr.params)
            (s0, ib), (sr, _) = adam_factors([lrs[names.index("sh0")], lrs[names.index("shN")]],
                                             o.betas, step)
            f[sh_off:sh_off + 3] = (s0, sr, ib)
        ci = tr.camera_index(it)
        n = len(self._vm_host)
        world_ci = [(ci - tr.rank + r) % n for r in range(self.W)] if self.gshard else [ci]
        b[512:512 + 64 * self.W].view(np.float32)[:] = self._vm_host[world_ci].reshape(-1)
        b[1024:1024 + 36 * self.W].view(np.float32)[:] = self._K_host[world_ci].reshape(-1)
        b[256:264].view(np.int64)[0] = ci
        if getattr(tr, "mcmc", False):
            b[264:272].view(np.int64)[0] = it
            b[272:276].view(np.float32)[0] = \
                0.0 if tr.strategy.is_refine_step(it) else tr.mcmc_scaler(it)
        if tr.model == "2dgs":  # rasterization_2dgs's torch.linalg.inv(viewmats), on the host
            b[1536:1536 + 64].view(np.float32)[:] = np.linalg.inv(
                self._vm_host[ci].astype(np.float64)).astype(np.float32).reshape(-1)
        if tr.max_steps:
            tr._set_means_lr(lrs[0])

    def _key_of(self, deg, stats):
        """What a capture is valid for: SH degree, the parameter tensors
        (their generation: a refine replaces them) and whether the step
        accumulates the strategy statistics."""
        tr = self.tr
        return (deg, tr.params["means"].shape[0], getattr(tr, "_param_gen", 0), stats)

    def _stats_at(self, it):
        st = self.tr.strategy
        if getattr(self.tr, "mcmc", False):
            return False  # MCMCStrategy keeps no statistics
        return st is None or it < st.refine_stop_iter

    def step(self, it):
        tr = self.tr
        deg = tr.sh_degree_at(it)
        stats = self._stats_at(it)
        key = self._key_of(deg, stats)
        if self.failed is not None:
            raise GraphCaptureError(self.failed)
        if self.graph is None or key != self.key:
            self._drain()
            if self.failed is not None:
                raise GraphCaptureError(self.failed)
            if self.key is not None and key[1] != self.key[1] and self.capacity is not None:
                # a refine changed the Gaussian count: grow the isect capacity
                # in proportion (an overflow would void and re-run the step)
                self.capacity = max(self.capacity,
                                    int(math.ceil(self.capacity * key[1] / self.key[1])))
            self.graph = None  # the old capture's pool holds the old tensors
            self._capture(deg, stats)
        if not self.vote:
            self._check(block=len(self.pending) >= self.lag)
        elif len(self.pending) >= self.lag:
            # several ranks: the oldest step exactly when `lag` are pending,
            # on every rank alike (a recovery is collective)
            self._check(block=True, one=True)
        if self.failed is not None:  # a recovery's re-capture failed: eager from here
            raise GraphCaptureError(self.failed)
        return self._issue(it)

    def _issue(self, it, ret=None):
        """Replay step `it` as the `issued`-th step; returns its loss: the
        loss-ring slot `issued % LOSS_RING` (written by the loss launch), or,
        without the ring, a copy of the graph's static loss (overwritten by
        the next replay; eager Trainer.step returns a fresh tensor per step as
        well).  `ret`: a redo of a voided step writes into the tensor already
        returned for it (_recover)."""
        k = self.issued  # this replay's fetch sees seq == k
        slot = k % self.RING
        ev = self._slot_ev[slot]
        if ev is not None:
            ev.synchronize()  # the step that used this slot RING steps ago is done
        t0 = time.perf_counter()
        self._fill(it, slot)
        self.graph.replay()
        self.tr.opt.step_count += 1
        if self.ring_loss:
            ret = self.loss_ring[k % self.LOSS_RING]
        elif ret is None:
            # (detached: a clone would keep the captured step's autograd
            # graph alive into the next capture)
            ret = self.loss.detach().clone()
        else:
            ret.copy_(self.loss)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self._slot_ev[slot] = ev
        self.pending.append((it, slot, ev, k, ret))
        self.issued += 1
        self.replays += 1
        self.host_s += time.perf_counter() - t0  # host work of the step, waits excluded
        return ret

    def _check(self, block=False, one=False):
        """Read the counts of finished steps; on an overflow, redo from there.
        `one`: the oldest pending step only."""
        while self.pending:
            it, slot, ev = self.pending[0][:3]
            if not ev.query():
                if not block:
                    return
                ev.synchronize()
            block = False
            n_written, _, over, n_total = (int(x) for x in self._out[slot])
            self.max_isects = max(self.max_isects, n_total)
            if over:
                self._recover()
                return
            self.pending.popleft()
            if one:
                return

    def _recover(self):
        """Every pending step from the first overflowed one was void (sticky
        flag): grow, re-capture, re-run them in order."""
        tr = self.tr
        torch.cuda.synchronize(self.dev)
        redo = [(it, k, ret) for it, _, _, k, ret in self.pending]
        for _, slot, _, _, _ in self.pending:
            self.max_isects = max(self.max_isects, int(self._out[slot][3]))
        self.pending.clear()
        tr.opt.step_count -= len(redo)  # their Adam steps did not happen
        # (a rank voided by another's overflow keeps at least its capacity)
        self.capacity = max(self.capacity or 0,
                            int(math.ceil(self.max_isects * self.headroom)) + 1)
        self.status.zero_()
        # the redo steps take the voided steps' sequence numbers, so each
        # step's loss lands in the slot (or tensor) already returned for it
        self.issued = redo[0][1]
        try:
            self._capture(tr.sh_degree_at(redo[0][0]), self._stats_at(redo[0][0]))
        except GraphCaptureError as e:
            # no graph any more: the voided steps run eagerly, in order, before
            # anything else (their losses into the tensors already returned),
            # and the trainer issues every later step eagerly (self.failed)
            self.failed = str(e)
            self.graph, self.key = None, None
            for it, _, ret in redo:
                loss = tr._eager_step(it)
                if getattr(tr, "mcmc", False) and not tr.strategy.is_refine_step(it):
                    tr.mcmc_noise(it)  # the replay's noise (a refine step's follows its refine)
                if ret is not None:
                    ret.copy_(loss.detach().reshape(ret.shape))
            return
        for it, k, ret in redo:
            assert self.issued == k
            self._issue(it, ret)
            self._check(block=True)

    def _drain(self):
        while self.pending and self.failed is None:
            self._check(block=True)

    def sync(self):
        """Wait for every issued step and settle its overflow check."""
        self._drain()
        torch.cuda.synchronize(self.dev)

    def release(self):
        """Settle the issued steps and destroy the captured graph.  A graph
        that captured RCCL collectives keeps their communicator's resources
        referenced until it is destroyed, and destroy_process_group waits for
        them (a test process hung there with the graph still alive): free the
        graph before the process group goes."""
        if self.graph is not None:
            self.sync()
            self.graph.reset()
            self.graph = None
        self.key = None
