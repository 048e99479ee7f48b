"""Communication for Gaussian-sharded rendering (the reference's
`rasterization(distributed=True)`, gsplat/rendering.py:298-494), over RCCL on
MI355X (torch.distributed "nccl" = RCCL, xGMI).

Same helper surface as gsplat/distributed.py:10-257:
    all_gather_int32, all_to_all_int32, all_gather_tensor_list,
    all_to_all_tensor_list (differentiable).
The many-to-many exchange of rows is one RCCL `all_to_all_single` over
contiguous buffers (on a fully connected xGMI node every peer pair has its
own link); on other backends (gloo: the CPU tests, and several ranks sharing
one GPU) explicit per-peer P2P transfers (`batch_isend_irecv`).  The backward
of an exchange is the exchange with input and output splits swapped.
"""

import contextlib
import math
import os
from contextlib import nullcontext as _nullcontext
from typing import List, Optional, Tuple, Union

import torch
import torch.distributed as dist
import torch.distributed.nn.functional as distF
from torch import Tensor


# ---- the process group of captured collectives ----------------------------
# While a HIP graph captures a training step (graph_step.GraphStep), its
# collectives run on a communicator that never issues eager work: RCCL's
# watchdog thread queries the end events of the eager collectives it still
# tracks, and a query of an event recorded on a stream that a capture has
# pulled in (the communicator's own stream, once a captured collective runs
# on it) is illegal -- a test process aborted that way.  Collectives issued
# during a capture are never tracked (torch does not enqueue them), so a
# group used ONLY inside captures gives the watchdog nothing to query there,
# by construction.  None: the default group.
_CAPTURE_PG = None


@contextlib.contextmanager
def capture_group(pg):
    """Route this module's collectives (the pair exchange, ShardedAdam while
    capturing) to `pg` inside the block."""
    global _CAPTURE_PG
    old, _CAPTURE_PG = _CAPTURE_PG, pg
    try:
        yield
    finally:
        _CAPTURE_PG = old


def current_capture_group():
    return _CAPTURE_PG


def new_capture_group():
    """A process group over every rank for captured collectives only (see
    _CAPTURE_PG).  Its communicator must exist before the capture without an
    eager collective on it: that needs the default group bound to a device
    (init_process_group(device_id=...)), which makes new_group connect
    eagerly.  Collective over the ranks (every rank creates its trainer's
    GraphStep in the same order)."""
    if dist.get_backend() == "nccl" and getattr(dist.distributed_c10d._get_default_group(),
                                                "bound_device_id", None) is None:
        raise RuntimeError("captured RCCL collectives need init_process_group(device_id=...) "
                           "(an eagerly connected communicator for the capture group)")
    return dist.new_group(list(range(dist.get_world_size())))


# ---- progress watchdog -------------------------------------------------------
class Watchdog:
    """gsplat_hip_watchdog_* (csrc/watchdog.cpp): a native thread that ends
    the process when no progress is reported within `timeout_s` -- printing
    the last reported state (rank, step, phase, capture / replay) to stderr
    and exiting with `exit_code` -- so that a collective one rank never joins
    ends a multi-GPU job with a diagnosis, not a silent hang (a collective
    replayed inside a HIP graph is invisible to RCCL's own timeout, and a
    host thread blocked in a HIP wait never returns to Python)."""

    def __init__(self, timeout_s: float, tag: str, exit_code: int = 3):
        from . import _lib
        self._lib = _lib
        self.timeout_s, self.tag, self.exit_code = float(timeout_s), tag, int(exit_code)
        self.armed = False

    def arm(self, state: str = "armed"):
        self._lib.call("gsplat_hip_watchdog_arm", self.timeout_s, self.tag.encode(),
                       self.exit_code)
        self.armed = True
        self.beat(state)

    def beat(self, state: str):
        if self.armed:
            self._lib.call("gsplat_hip_watchdog_beat", state.encode(errors="replace"))

    def fallback(self, fd: int, text: Optional[str], exit_code: int = 0):
        """On expiry also write `text` to `fd` and exit with `exit_code`."""
        self._lib.call("gsplat_hip_watchdog_set_fallback", int(fd) if text is not None else -1,
                       (text or "").encode(), int(exit_code))

    def disarm(self):
        if self.armed:
            self._lib.call("gsplat_hip_watchdog_disarm")
            self.armed = False


def all_gather_int32(world_size: int, value: Union[int, Tensor],
                     device: Optional[torch.device] = None) -> List:
    """One 32-bit integer from every rank (gsplat/distributed.py:10-52)."""
    if world_size == 1:
        return [value]
    if isinstance(value, int):
        assert device is not None, "device is required for scalar input"
        t = torch.tensor(value, dtype=torch.int, device=device)
    else:
        t = value
    collected = torch.empty(world_size, dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(collected, t.reshape(1))
    return collected.tolist() if isinstance(value, int) else list(collected.unbind())


def _exchange(send: List[Tensor], recv: List[Tensor]) -> None:
    """recv[j] <- rank j's send[me]; send[j] -> rank j (P2P, one op per peer).
    gloo with GPU tensors (several ranks sharing one GPU in the tests) goes
    through host copies: gloo's P2P moves host memory only."""
    me = dist.get_rank()
    if send and send[0].is_cuda and dist.get_backend() == "gloo":
        hs = [t.cpu() for t in send]
        hr = [torch.empty(r.shape, dtype=r.dtype) for r in recv]
        _exchange(hs, hr)
        for r, h in zip(recv, hr):
            r.copy_(h)
        return
    recv[me].copy_(send[me])
    ops = []
    for j in range(len(send)):
        if j == me:
            continue
        if recv[j].numel():
            ops.append(dist.P2POp(dist.irecv, recv[j].contiguous(), j))
        if send[j].numel():
            ops.append(dist.P2POp(dist.isend, send[j].contiguous(), j))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()


def all_to_all_int32(world_size: int, values: List[Union[int, Tensor]],
                     device: Optional[torch.device] = None) -> List:
    """Exchange one 32-bit integer per rank pair (gsplat/distributed.py:55-99)."""
    if world_size == 1:
        return values
    assert len(values) == world_size, "The length of values should be equal to world_size"
    if any(isinstance(v, int) for v in values):
        assert device is not None, "device is required for scalar input"
    send = [(torch.tensor([v], dtype=torch.int, device=device) if isinstance(v, int)
             else v.reshape(1)) for v in values]
    recv = [torch.empty_like(s) for s in send]
    _exchange(send, recv)
    return [r.item() if isinstance(v, int) else r.reshape(())
            for r, v in zip(recv, values)]


def all_gather_tensor_list(world_size: int, tensor_list: List[Tensor]) -> List[Tensor]:
    """Concatenate every rank's tensors along dim 0, differentiably
    (gsplat/distributed.py:102-167)."""
    if world_size == 1:
        return tensor_list
    N = len(tensor_list[0])
    for t in tensor_list:
        assert len(t) == N, "All tensors should have the same first dimension size"
    data = torch.cat([t.reshape(N, -1) for t in tensor_list], dim=-1)
    sizes = [t.numel() // N for t in tensor_list]
    if data.requires_grad:
        collected = distF.all_gather(data)
    else:
        collected = [torch.empty_like(data) for _ in range(world_size)]
        dist.all_gather(collected, data)
    collected = torch.cat(collected, dim=0)
    return [o.reshape(-1, *t.shape[1:]) for o, t in
            zip(torch.split(collected, sizes, dim=-1), tensor_list)]


# ---- measurement only (bench.py --gshard-emulate W): one process stands in
# for rank 0 of a W-rank Gaussian-sharded job, to time that rank's compute on
# one GPU.  Its exchanges take their peers' rows from stand-ins instead of
# RCCL: forward, the rows each peer's own render would send to rank 0
# (recorded once by running that peer's render up to its exchange, `record`),
# backward, rank 0's own gradient block in every peer's place (same sizes).
# The stand-ins are concatenated on the device, so the rows are copied but
# no link is crossed: the exchange's xGMI time is not part of the measurement.
class _Recorded(Exception):
    """Raised by a recording render once its rows for rank 0 are kept."""


class Emulation:
    def __init__(self, world: int):
        self.world, self.rank = int(world), 0
        self.recording = False
        self.standins = {}  # dtype -> {peer rank: rows for rank 0}

    def record(self, rank: int, render) -> None:
        """Run peer `rank`'s render (a callable) up to its float exchange and
        keep the rows it sends to rank 0."""
        self.rank, self.recording = int(rank), True
        try:
            with torch.no_grad():
                render()
        except _Recorded:
            pass
        finally:
            self.rank, self.recording = 0, False

    def rows(self, data: Tensor, splits: List[int], out_splits: List[int], backward: bool):
        own = data[:splits[0]]  # the block rank 0 sends to itself
        if self.recording:
            self.standins.setdefault(data.dtype, {})[self.rank] = own.clone()
            if data.dtype == torch.float32:
                raise _Recorded()
            return data.new_zeros((sum(out_splits),) + data.shape[1:])
        parts = [own]
        for j in range(1, self.world):
            if backward:
                assert out_splits[j] == own.shape[0], (out_splits, own.shape)
                parts.append(own)
            else:
                blk = self.standins[data.dtype][j]
                assert blk.shape == (out_splits[j],) + data.shape[1:], (blk.shape, out_splits)
                parts.append(blk)
        return torch.cat(parts, dim=0)


EMULATION: Optional[Emulation] = None


def rank_world() -> Tuple[int, int]:
    """(rank, world size) of the process group, or of the emulated job."""
    if EMULATION is not None:
        return EMULATION.rank, EMULATION.world
    return dist.get_rank(), dist.get_world_size()


def _all_to_all_rows(data: Tensor, splits: List[int], out_splits: List[int],
                     backward: bool = False) -> Tensor:
    """Rows data[sum(splits[:j]) : ...] to rank j; rank j's rows for me, in
    rank order.  RCCL: one all_to_all_single over contiguous buffers (the
    collective xGMI is built for, no per-peer concat); other backends: the
    per-peer P2P exchange."""
    data = data.contiguous()
    if EMULATION is not None:
        return EMULATION.rows(data, splits, out_splits, backward)
    if data.is_cuda and dist.get_backend() == "nccl":
        out = data.new_empty((sum(out_splits),) + data.shape[1:])
        dist.all_to_all_single(out, data, output_split_sizes=out_splits,
                               input_split_sizes=splits, group=_CAPTURE_PG)
        return out
    send = list(data.split(splits, dim=0))
    recv = [data.new_empty((n,) + data.shape[1:]) for n in out_splits]
    _exchange(send, recv)
    return torch.cat(recv, dim=0)


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, splits, out_splits):
        ctx.splits, ctx.out_splits = splits, out_splits
        return _all_to_all_rows(data, splits, out_splits)

    @staticmethod
    def backward(ctx, grad):
        return _all_to_all_rows(grad, ctx.out_splits, ctx.splits, backward=True), None, None


class _ExchangePairs(torch.autograd.Function):
    """The projected pairs of a Gaussian-sharded render with one camera per
    rank, in ONE exchange: rank r sends camera j's rows of its shard to rank
    j and receives every rank's rows for its own camera.  Per destination the
    send buffer is field-major -- radii (int32 bits), means2d, depths, conics,
    opacities, colours, each a contiguous run of the shard's rows -- so
    packing is one concatenation of large contiguous runs and unpacking one
    per field, and every output is contiguous (the row-interleaved packing of
    all_to_all_tensor_list and the column views it hands out cost ~0.2 ms of
    copies per step at M2).  Backward: the gradient fields packed per source
    rank, the reverse exchange, camera-major views of the received runs."""

    @staticmethod
    def forward(ctx, n_world, radii, *fields):
        C, Nr = fields[0].shape[:2]
        W = len(n_world)
        assert C == W and radii.dtype == torch.int32 and radii.shape[:2] == (C, Nr)
        shapes = [tuple(f.shape[2:]) for f in fields]
        widths = [math.prod(sh) for sh in shapes]
        rw = math.prod(radii.shape[2:])
        tot = rw + sum(widths)
        send = torch.cat([radii.reshape(C, -1).view(torch.float32)] +
                         [f.reshape(C, -1) for f in fields], dim=1)  # [C, Nr * tot]
        recv = _all_to_all_rows(send.reshape(-1), [Nr * tot] * C, [n * tot for n in n_world])
        ntot = sum(n_world)
        cols = [rw] + widths
        K = len(cols)
        # one split into every (source, field) run, one cat per field: few
        # host-side ops (the step is eager; slicing run by run cost ~0.1 ms
        # of host time per render)
        runs = recv.split([n * w for n in n_world for w in cols])
        outs = [torch.cat(runs[k::K]) for k in range(K)]
        r_out = outs[0].view(torch.int32).view(1, ntot, *radii.shape[2:])
        f_out = [o.view(1, ntot, *sh) for o, sh in zip(outs[1:], shapes)]
        ctx.n_world, ctx.Nr, ctx.shapes, ctx.widths = list(n_world), Nr, shapes, widths
        ctx.dtype, ctx.device = fields[0].dtype, fields[0].device
        ctx.mark_non_differentiable(r_out)
        return (r_out, *f_out)

    @staticmethod
    def backward(ctx, _g_radii, *grads):
        n_world, Nr, shapes, widths = ctx.n_world, ctx.Nr, ctx.shapes, ctx.widths
        W, ntot, tot = len(n_world), sum(n_world), sum(widths)
        # a field without a gradient sends zeros; so does a loss that reaches
        # none of them -- every rank must still join the reverse all_to_all
        ref = next((g for g in grads if g is not None), None)
        if ref is None:
            ref = torch.zeros(0, dtype=ctx.dtype, device=ctx.device)
        # [field][source rank] runs of each gradient field, flat
        runs = [(g if g is not None else ref.new_zeros((1, ntot) + sh)).reshape(-1)
                .split([n * w for n in n_world]) for g, sh, w in zip(grads, shapes, widths)]
        send = torch.cat([r[i] for i in range(W) for r in runs])
        recv = _all_to_all_rows(send, [n * tot for n in n_world], [Nr * tot] * W,
                                backward=True).view(W, Nr * tot)
        out, off = [], 0
        for sh, w in zip(shapes, widths):
            out.append(recv[:, Nr * off:Nr * (off + w)].reshape(W, Nr, *sh))
            off += w
        return (None, None, *out)


def exchange_pairs(n_world: List[int], radii: Tensor, means2d: Tensor, depths: Tensor,
                   conics: Tensor, opacities: Tensor, colors: Tensor):
    """One camera per rank: [W, N_r, ...] pairs of this shard in every rank's
    camera -> [1, sum N_i, ...] pairs of every shard in this rank's camera,
    rank order (_ExchangePairs).  Returns radii, means2d, depths, conics,
    opacities, colors."""
    return _ExchangePairs.apply([int(n) for n in n_world], radii.contiguous(), means2d, depths,
                                conics, opacities, colors)


def all_to_all_tensor_list(world_size: int, tensor_list: List[Tensor],
                           splits: List[Union[int, Tensor]],
                           output_splits: Optional[List[Union[int, Tensor]]] = None
                           ) -> List[Tensor]:
    """Split every tensor along dim 0 by `splits` and exchange the pieces,
    differentiably (gsplat/distributed.py:170-257)."""
    if world_size == 1:
        return tensor_list
    N = len(tensor_list[0])
    for t in tensor_list:
        assert len(t) == N, "All tensors should have the same first dimension size"
    assert len(splits) == world_size, "The length of splits should be equal to world_size"
    data = torch.cat([t.reshape(N, -1) for t in tensor_list], dim=-1)
    sizes = [t.numel() // N for t in tensor_list]
    if output_splits is None:
        output_splits = all_to_all_int32(world_size, splits, device=data.device)
    splits = [int(s) for s in splits]
    output_splits = [int(s) for s in output_splits]
    collected = _AllToAll.apply(data, splits, output_splits)
    return [o.reshape(-1, *t.shape[1:]) for o, t in
            zip(torch.split(collected, sizes, dim=-1), tensor_list)]


# ------------------------------------------- per-camera data parallelism --

def _adam_torch(params, grads, exp_avgs, exp_avg_sqs, lrs, betas, eps, step, aux=None,
                modes=None):
    """torch restatement of csrc/adam.hip's update (same operation order, the
    gradient transforms of gsplat_hip_adam_step_ex included), for running
    ShardedAdam's collectives on the CPU (gloo tests)."""
    b1, b2 = betas
    bc1, bc2 = 1.0 - b1 ** step, 1.0 - b2 ** step
    aux = aux or [None] * len(params)
    modes = modes or [0] * len(params)
    for p, g, m, v, lr, a, md in zip(params, grads, exp_avgs, exp_avg_sqs, lrs, aux, modes):
        g = torch.zeros_like(p) if g is None else g
        if md == 1:
            g = g + a
        elif md == 2:
            g = g * a
        elif md == 3:
            g = g * (1.0 - a) * a
        m.add_((1.0 - b1) * (g - m))
        v.mul_(b2).add_((1.0 - b2) * g * g)
        p.sub_((lr / bc1) * m / (v.sqrt() * (1.0 / math.sqrt(bc2)) + eps))


class ShardedAdam:
    """Adam for per-camera data parallelism with the optimizer state sharded
    over the ranks: per parameter, the summed gradient is reduce-scattered
    (each rank receives the sum of its 1/world_size of the rows), each rank
    updates its rows only, and the updated rows are all-gathered back into
    every replica.  Same bytes on the wire as one all-reduce of the gradients
    (a ring all-reduce is a reduce-scatter plus an all-gather), but the Adam
    pass and its 2 x 4 B/element moment state shrink to 1/world_size per rank.

    Rows are split in multiples of 4 (16-B aligned shards for the fused
    kernel); the < 4 * world_size remainder rows are all-reduced and updated
    redundantly on every rank.  Collectives run on the default group.  `update`
    is the Adam kernel (csrc/adam.hip by default).

    `groups` (lists of parameter indices, in issue order; default one group)
    pipelines the step: per group, its reduce-scatters are issued from the
    current stream (after the backward), and on a side stream the group's Adam
    waits for them, updates the shards and issues the group's all-gathers.  So
    the RCCL stream runs RS(g0), AG(g0), RS(g1), AG(g1) ...: the trainer puts
    the geometry first (the next projection needs it, 44 B/Gaussian) and the SH
    rows last (192 B/Gaussian, needed only by the colours after the next
    isect), and neither the host nor the compute stream waits for any of it.

    `group_pgs` gives each group its own process group (communicator), so the
    groups' collectives do not queue behind each other: the trainer issues
    the SH group's reduce-scatter from a gradient hook while the backward is
    still running (`reduce_early`) on one communicator, and the geometry's
    after the backward on another -- the small, latency-critical geometry
    exchange never waits for the 4x larger SH one.

    `step(xform=...)` folds the trainer's gradient transforms into the update
    (gsplat_hip_adam_step_ex): the activation VJPs (modes 2 / 3) are linear
    in the incoming gradient, so that gradient is what is reduce-scattered
    and the VJP is applied to the summed shard in-register (its `aux`, the
    activation, is replicated and sliced like the parameter); a second
    gradient term (mode 1) is summed locally before the reduction.
    """

    def __init__(self, params, lrs, betas=(0.9, 0.999), eps=1e-8, update=None, groups=None,
                 group_pgs=None, emulate_world=None):
        self.params = list(params)
        self.lrs = [float(x) for x in lrs]
        self.betas, self.eps = betas, eps
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        # a group of one rank exchanges nothing: the collectives are skipped
        # (the shard is the gradient itself, the rows are updated in place)
        # (GSPLAT_HIP_DP_SOLO=0: the collectives on a one-rank group as well --
        # the RCCL path of an N > 1 job, checked on one GPU by the tests)
        self.solo = self.world == 1 and os.environ.get("GSPLAT_HIP_DP_SOLO", "1") != "0"
        if emulate_world:
            # measurement only (bench.py --dp-emulate): on ONE rank, shard the
            # rows as `emulate_world` ranks would and update rank 0's share --
            # the per-rank optimizer work of that world size, without its
            # collectives; the other shards are left stale
            assert self.solo, "emulate_world needs a 1-rank group"
            self.world = int(emulate_world)
        if update is None:
            from .losses import adam_groups
            update = adam_groups
        self.update = update
        self.step_count = 0
        w, r = self.world, self.rank
        self.layout = []  # (row floats, shard rows q, main floats w*q*row, total floats)
        for p in self.params:
            assert p.is_contiguous() and p.dtype == torch.float32
            row = p[0].numel() if p.dim() > 0 and p.shape[0] > 0 else 1
            q = (p.shape[0] // (4 * w)) * 4
            self.layout.append((row, q, w * q * row, p.numel()))
        dev = self.params[0].device
        z = lambda n: torch.zeros(n, device=dev)  # noqa: E731
        self.m = [z(q * row) for row, q, _, _ in self.layout]
        self.v = [z(q * row) for row, q, _, _ in self.layout]
        self.m_tail = [z(tot - main) for _, _, main, tot in self.layout]
        self.v_tail = [z(tot - main) for _, _, main, tot in self.layout]
        self.g_shard = [torch.empty(0 if self.solo else q * row, device=dev)
                        for row, q, _, _ in self.layout]
        self.order = sorted(range(len(self.params)), key=lambda i: -self.params[i].numel())
        self.groups = [list(g) for g in groups] if groups else [list(self.order)]
        assert sorted(i for g in self.groups for i in g) == list(range(len(self.params))), \
            self.groups
        self.group_pgs = list(group_pgs) if group_pgs else [None] * len(self.groups)
        assert len(self.group_pgs) == len(self.groups)
        self._early = {}  # group index -> (flats, works) issued by reduce_early
        self._pending = {}  # parameter index -> all-gather still in flight
        # parameter index -> event after its group's update on the side stream
        # (tail rows and parameters too short for a shard are updated there
        # and have no all-gather to wait on)
        self._updated = {}
        # Adam + all-gather issue stream (CUDA only; gloo runs them inline)
        self.side = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        # set while a HIP graph captures the step (graph_step.GraphStep): every
        # collective on the default group, issued and waited for in order on
        # the capturing stream -- no side stream, no second communicator, no
        # early SH reduce-scatter (a capture with them crashed in
        # hipStreamEndCapture on a one-rank RCCL group); the graph's replay
        # has no host gaps to hide anyway
        self.capturing = False

    def wait(self, indices=None):
        """Order the current stream after the deferred all-gathers of these
        parameters (all when None); no host synchronisation."""
        for i in (set(self._pending) | set(self._updated)) if indices is None else indices:
            ev = self._updated.pop(i, None)
            if ev is not None:
                torch.cuda.current_stream(self.params[i].device).wait_event(ev)
            wk = self._pending.pop(i, None)
            if wk is not None:
                wk.wait()

    def _shard(self, i, flat):
        row, q, _, _ = self.layout[i]
        return flat[self.rank * q * row:(self.rank + 1) * q * row]

    def _issue_reduce(self, gi, grads):
        """Reduce-scatter (main rows) and all-reduce (remainder rows) of group
        gi's gradients on its process group, issued from the current stream."""
        # capturing: in order on the capturing stream, on the capture-only
        # group (graph_step; the default group during the capture's warm-up)
        pg = _CAPTURE_PG if self.capturing else self.group_pgs[gi]
        flats, works = {}, []
        for i in sorted(self.groups[gi], key=lambda i: -self.params[i].numel()):
            g = grads.get(i)
            gf = (torch.zeros_like(self.params[i]) if g is None else g).contiguous().view(-1)
            flats[i] = gf
            if self.side is not None and not self.capturing:  # tail rows read on the side stream
                gf.record_stream(self.side)
            _, _, main, tot = self.layout[i]
            if self.solo:
                continue  # the shard is this gradient's own rows (_update_group)
            if main:
                works.append(dist.reduce_scatter_tensor(self.g_shard[i], gf[:main], group=pg,
                                                        async_op=True))
            if tot > main:
                works.append(dist.all_reduce(gf[main:], group=pg, async_op=True))
        return flats, works

    def _grads(self, grp, xform):
        out = {}
        for i in grp:
            if xform and i in xform:
                g, a, mode = xform[i]
                out[i] = g + a if mode == 1 else g  # modes 2 / 3: applied after the reduction
            else:
                out[i] = self.params[i].grad
        return out

    @torch.no_grad()
    def reduce_early(self, gi, xform=None):
        """Issue group gi's reductions now (from a gradient hook, while the
        rest of the backward is still being queued); the next step() only
        waits for them.  Stream order only, no host synchronisation."""
        if self.capturing:
            return  # step() issues it, in order
        if gi not in self._early:
            self._early[gi] = self._issue_reduce(gi, self._grads(self.groups[gi], xform))

    def launch_plan(self):
        """The parameter indices of each Adam launch of step(), in launch
        order: per group its shard rows, then its remainder rows.  A captured
        step's device-side factors (`hyper`) are laid out in this order."""
        plan = []
        for grp in self.groups:
            for sel in ([i for i in grp if self.layout[i][2]],
                        [i for i in grp if self.layout[i][3] > self.layout[i][2]]):
                if sel:
                    plan.append(sel)
        return plan

    @torch.no_grad()
    def step(self, defer_gather=False, xform=None, hyper=None, void=None):
        """defer_gather: leave the all-gathers in flight; the caller orders
        each parameter's next use after `wait([i])` (stream order only).
        xform: {index: (grad, aux, mode)} as FusedAdam.step (see the class
        docstring for where each mode is applied).  hyper / void: the
        captured step's device-side Adam factors (adam_factors of every
        launch of launch_plan(), in its order) and void-step flag; step_count
        is then the caller's business (graph_step.GraphStep)."""
        self.wait()
        if hyper is None:
            self.step_count += 1
        self._hyper = None if hyper is None else [hyper, 0, void]
        side = None if self.capturing else self.side
        for gi, grp in enumerate(self.groups):
            if gi in self._early:
                flats, works = self._early.pop(gi)
            else:
                flats, works = self._issue_reduce(gi, self._grads(grp, xform))
            if side is not None:  # the side stream starts after everything queued so far
                side.wait_stream(torch.cuda.current_stream(side.device))
            with (torch.cuda.stream(side) if side is not None else _nullcontext()):
                for wk in works:  # the side stream (gloo: the host) waits
                    wk.wait()
                self._update_group(grp, flats, xform)
                if side is not None:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    for i in grp:
                        self._updated[i] = ev
                # issued from the side stream: RCCL waits for this Adam only.
                # RCCL gathers in place (the send buffer is this rank's slice
                # of the output, NCCL's in-place all-gather); gloo gets a copy
                for i in sorted(grp, key=lambda i: self.params[i].numel()):
                    _, _, main, _ = self.layout[i]
                    if main and not self.solo:
                        full = self.params[i].data.view(-1)[:main]
                        mine = self._shard(i, full)
                        self._pending[i] = dist.all_gather_into_tensor(
                            full, mine if full.is_cuda else mine.clone(),
                            group=_CAPTURE_PG if self.capturing else self.group_pgs[gi],
                            async_op=True)
        if not defer_gather:
            self.wait()

    def _dev(self, n):
        """kwargs of the next launch's device-side factors (captured step)."""
        h = getattr(self, "_hyper", None)
        if h is None:
            return {}
        hyper, off, void = h
        h[1] = off + 2 * n
        return dict(hyper=hyper[off:off + 2 * n], skip=void)

    def _update_group(self, grp, flats, xform=None):
        def tx(i):  # (aux, mode) of a post-reduction transform, else (None, 0)
            if xform and i in xform and xform[i][2] in (2, 3):
                return xform[i][1].reshape(-1), xform[i][2]
            return None, 0
        idx = [i for i in grp if self.layout[i][2]]
        if idx:
            aux = [tx(i)[0] for i in idx]
            # one rank: the reduce-scatter's output is the gradient's own rows
            gsh = [self._shard(i, flats[i]) if self.solo else self.g_shard[i] for i in idx]
            self.update([self._shard(i, self.params[i].data.view(-1)) for i in idx],
                        gsh, [self.m[i] for i in idx],
                        [self.v[i] for i in idx], [self.lrs[i] for i in idx], self.betas,
                        self.eps, self.step_count,
                        aux=[None if a is None else self._shard(i, a) for i, a in zip(idx, aux)],
                        modes=[tx(i)[1] for i in idx], **self._dev(len(idx)))
        tails = [i for i in grp if self.layout[i][3] > self.layout[i][2]]
        if tails:
            aux = [tx(i)[0] for i in tails]
            self.update([self.params[i].data.view(-1)[self.layout[i][2]:] for i in tails],
                        [flats[i][self.layout[i][2]:] for i in tails],
                        [self.m_tail[i] for i in tails], [self.v_tail[i] for i in tails],
                        [self.lrs[i] for i in tails], self.betas, self.eps, self.step_count,
                        aux=[None if a is None else a[self.layout[i][2]:]
                             for i, a in zip(tails, aux)],
                        modes=[tx(i)[1] for i in tails], **self._dev(len(tails)))

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def full_state(self):
        """[(exp_avg, exp_avg_sq)] per parameter as full tensors shaped like it:
        the shards all-gathered (the replicated tail rows appended).  For the
        optimizer-state surgery of a densification step (every rank gets the
        same tensors)."""
        assert self.world == dist.get_world_size(), "full_state: not with emulate_world"
        self.wait()
        out = []
        for i, p in enumerate(self.params):
            _, _, main, tot = self.layout[i]
            pair = []
            for shard, tail in ((self.m[i], self.m_tail[i]), (self.v[i], self.v_tail[i])):
                full = torch.empty(tot, device=p.device, dtype=p.dtype)
                if main:
                    dist.all_gather_into_tensor(full[:main], shard)
                full[main:] = tail
                pair.append(full.view_as(p))
            out.append(tuple(pair))
        return out

    @torch.no_grad()
    def load_full_state(self, moments, step_count):
        """Inverse of full_state for this optimizer's (new) parameters: keep
        this rank's shard and the tail rows of each full moment tensor."""
        self.step_count = int(step_count)
        for i, (m, v) in enumerate(moments):
            _, _, main, _ = self.layout[i]
            for full, shard, tail in ((m, self.m[i], self.m_tail[i]), (v, self.v[i], self.v_tail[i])):
                f = full.reshape(-1)
                if main:
                    shard.copy_(self._shard(i, f[:main]))
                tail.copy_(f[main:])

    @torch.no_grad()
    def zero_moments(self, i):
        """Zero both moments of parameter i (reset_opa's optimizer state)."""
        for t in (self.m[i], self.v[i], self.m_tail[i], self.v_tail[i]):
            t.zero_()
