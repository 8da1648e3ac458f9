"""One-time replica initialisation: rank 0's parameters and buffers everywhere.

This is DDP's constructor broadcast (reference `tools/train.py:86`, SURVEY
collective site C2) without DDP.  It covers EVERYTHING in the distiller's
state -- student and distiller-module parameters (the flat buffer), teacher
parameters (random-init teachers in benchmarks; a checkpoint-loaded teacher
is already identical and pays one cheap broadcast), BN running statistics,
CRD memory banks and normaliser constants, OFD margins -- so the ranks start
bit-identical whatever each rank's RNG state was.

Messages are coalesced per dtype into a handful of flat buffers (a few tens
of MB for the north-star pair), so this is a few large RCCL broadcasts over
xGMI rather than one per tensor.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import is_dist

# coalescing cap per message (bytes): big enough to amortise latency, small
# enough not to double peak memory for ImageNet-size CRD banks
_CHUNK_BYTES = 256 << 20


def _unique_storage_tensors(module, exclude_ptrs):
    seen = set(exclude_ptrs)
    out = []
    for t in list(module.parameters()) + list(module.buffers()):
        if t is None or t.numel() == 0:
            continue
        key = (t.data_ptr(), t.numel(), t.dtype)
        if t.data_ptr() in exclude_ptrs or key in seen:
            continue
        seen.add(key)
        out.append(t)
    return out


@torch.no_grad()
def _broadcast_coalesced(tensors, src, group=None):
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    n_calls = 0
    for (dt, dev), ts in by_dtype.items():
        i = 0
        while i < len(ts):
            chunk, nbytes = [], 0
            while i < len(ts) and (not chunk or nbytes + ts[i].numel() * ts[i].element_size() <= _CHUNK_BYTES):
                chunk.append(ts[i])
                nbytes += ts[i].numel() * ts[i].element_size()
                i += 1
            if len(chunk) == 1 and chunk[0].is_contiguous():
                dist.broadcast(chunk[0].data, src, group=group)
            else:
                flat = torch.cat([c.detach().reshape(-1) for c in chunk])
                dist.broadcast(flat, src, group=group)
                off = 0
                for c in chunk:
                    n = c.numel()
                    c.data.copy_(flat[off:off + n].view_as(c))
                    off += n
            n_calls += 1
    return n_calls


@torch.no_grad()
def broadcast_initial_state(module, flat=None, src: int = 0, group=None) -> int:
    """Make every rank's ``module`` state equal to rank ``src``'s.

    ``flat``: the :class:`~..engine.optim.FlatParams` whose buffer backs the
    learnable parameters; it is broadcast as ONE message and the views it
    backs are skipped.  Returns the number of collectives issued (0 when
    not distributed).
    """
    if not is_dist():
        return 0
    calls = 0
    skip = set()
    if flat is not None:
        dist.broadcast(flat.data, src, group=group)
        calls += 1
        skip = {p.data_ptr() for p in flat.params}
    calls += _broadcast_coalesced(_unique_storage_tensors(module, skip), src, group)
    return calls


@torch.no_grad()
def state_checksum(module, flat=None, buffers: bool = True) -> torch.Tensor:
    """Order-sensitive float64 checksum of all parameters (and buffers) (tests).

    Student BN running statistics legitimately differ between ranks during
    training (each rank normalises its own shard, as under DDP, and rank 0's
    are broadcast before evaluation), so compare with ``buffers=False``
    mid-training."""
    dev = flat.data.device if flat is not None else next(module.parameters()).device
    acc = torch.zeros(2, dtype=torch.float64, device=dev)
    skip = {p.data_ptr() for p in flat.params} if flat is not None else set()
    if buffers:
        rest = _unique_storage_tensors(module, skip)
    else:
        rest = [p for p in module.parameters() if p.data_ptr() not in skip]
    ts = ([flat.data] if flat is not None else []) + rest
    for k, t in enumerate(ts):
        v = t.detach().reshape(-1).double()
        acc[0] += v.sum()
        w = torch.arange(v.numel(), device=v.device, dtype=torch.float64).remainder(89).add_(k + 1)
        acc[1] += (v * w).sum()
    return acc
