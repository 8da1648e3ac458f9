"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

Reads the torchrun environment correctly -- ``RANK`` is the global rank and
``LOCAL_RANK`` picks the device (the reference passes ``LOCAL_RANK`` as the
global rank, so multi-node runs collide: SURVEY D10).  Backend ``auto`` is
``nccl`` (= RCCL on ROCm) when GPUs are visible and ``gloo`` otherwise, which
is how every distributed test runs on CPU.  An explicit timeout is always set
and RCCL async error handling is enabled so a dead peer aborts the job
instead of hanging it.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_INFO = DistInfo()


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_distributed(backend: str = "auto", timeout_s: float = 600.0, device: str = "auto") -> DistInfo:
    """Initialise from torchrun env vars; a no-op (world 1) without them."""
    global _INFO
    world = _env_int("WORLD_SIZE", 1)
    rank = _env_int("RANK", _env_int("LOCAL_RANK", 0))
    local = _env_int("LOCAL_RANK", rank)
    use_gpu = torch.cuda.device_count() > 0 if device == "auto" else device == "cuda"
    if use_gpu:
        n = torch.cuda.device_count()
        torch.cuda.set_device(local % n)
        dev = torch.device("cuda", local % n)
    else:
        dev = torch.device("cpu")
    if backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
            opts = nccl_options()
            if opts is not None:
                kw["pg_options"] = opts
        try:
            dist.init_process_group(**kw)
        except TypeError:  # older torch without device_id
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    _INFO = DistInfo(rank, local, world, backend if world > 1 else "none", dev)
    os.environ["IS_MASTER_NODE"] = "1" if rank == 0 else "0"
    return _INFO


def nccl_options():
    """RCCL process-group options: the collectives run on HIGH-priority
    internal streams, so a bucket's all-reduce is dispatched ahead of the
    teacher / student kernels queued on the same device (docs/DESIGN.md 4).
    None when this torch build has no ProcessGroupNCCL."""
    pg = getattr(dist, "ProcessGroupNCCL", None)
    if pg is None or not hasattr(pg, "Options"):
        return None
    o = pg.Options()
    o.is_high_priority_stream = True
    return o


def info() -> DistInfo:
    return _INFO


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def get_rank() -> int:
    return dist.get_rank() if is_dist() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def get_local_rank() -> int:
    return _INFO.local_rank


def is_master() -> bool:
    return get_rank() == 0


def barrier() -> None:
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def destroy() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
