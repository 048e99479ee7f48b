"""Communication for Gaussian-sharded rendering (the reference's
`rasterization(distributed=True)`, gsplat/rendering.py:298-494), over RCCL on
MI355X (torch.distributed "nccl" = RCCL, xGMI).

Same helper surface as gsplat/distributed.py:10-257:
    all_gather_int32, all_to_all_int32, all_gather_tensor_list,
    all_to_all_tensor_list (differentiable).
The many-to-many exchange is written as explicit per-peer P2P transfers
(`batch_isend_irecv`): on a fully connected xGMI node every peer pair has its
own link, so the exchange is one transfer per link; the same code runs over
gloo on the CPU for the tests.  The backward of an exchange is the exchange
with input and output splits swapped.
"""

from typing import List, Optional, Union

import torch
import torch.distributed as dist
import torch.distributed.nn.functional as distF
from torch import Tensor


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
    """recv[j] <- rank j's send[me]; send[j] -> rank j (P2P, one op per peer)."""
    me = dist.get_rank()
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


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, splits, out_splits):
        ctx.splits, ctx.out_splits = splits, out_splits
        send = list(data.split(splits, dim=0))
        recv = [data.new_empty((n,) + data.shape[1:]) for n in out_splits]
        _exchange(send, recv)
        return torch.cat(recv, dim=0)

    @staticmethod
    def backward(ctx, grad):
        grad = grad.contiguous()
        send = list(grad.split(ctx.out_splits, dim=0))
        recv = [grad.new_empty((n,) + grad.shape[1:]) for n in ctx.splits]
        _exchange(send, recv)
        return torch.cat(recv, dim=0), None, None


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
