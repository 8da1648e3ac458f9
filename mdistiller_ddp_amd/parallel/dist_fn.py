"""Collective helpers with the reference's names and semantics
(`mdistiller/utils/dist_fn.py:6-41`): ``broadcast``, ``scatter``,
``gather`` (= all_gather + cat along dim 0) and ``reduce`` (= all_reduce, SUM
by default; ``"avg"`` divides by world size so it also works on gloo, which
has no AVG op).  All are identities when not distributed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import is_dist, get_world_size


def broadcast(tensor: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_dist():
        dist.broadcast(tensor, src)
    return tensor


def scatter(tensor: torch.Tensor, src: int = 0, dim: int = 0) -> torch.Tensor:
    """Split ``tensor`` (valid on ``src``) into world chunks; return own chunk."""
    if not is_dist():
        return tensor
    ws = get_world_size()
    chunks = list(tensor.chunk(ws, dim=dim))
    out = torch.empty_like(chunks[0])
    dist.scatter(out, [c.contiguous() for c in chunks] if dist.get_rank() == src else None, src=src)
    return out


def gather(tensor: torch.Tensor, dim: int = 0) -> torch.Tensor:
    if not is_dist():
        return tensor
    out = [torch.empty_like(tensor) for _ in range(get_world_size())]
    dist.all_gather(out, tensor.contiguous())
    return torch.cat(out, dim=dim)


def reduce(tensor: torch.Tensor, op: str | dist.ReduceOp = "sum") -> torch.Tensor:
    if not is_dist():
        return tensor
    avg = False
    if isinstance(op, str):
        avg = op.lower() in ("avg", "mean")
        op = dist.ReduceOp.SUM
    elif op == dist.ReduceOp.AVG and dist.get_backend() != "nccl":
        avg, op = True, dist.ReduceOp.SUM
    dist.all_reduce(tensor, op=op)
    if avg:
        tensor.div_(get_world_size())
    return tensor
