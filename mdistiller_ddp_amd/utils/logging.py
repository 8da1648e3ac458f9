"""Console / file logging helpers (reference `engine/utils.py:73-80`)."""
from __future__ import annotations

import os
import sys

_COLORS = {"INFO": 36, "TRAIN": 32, "EVAL": 31, "WARN": 33, "PERF": 35}


def log_msg(msg: str, mode: str = "INFO") -> str:
    color = _COLORS.get(mode, 37)
    if not sys.stdout.isatty() and os.environ.get("MDA_FORCE_COLOR", "0") != "1":
        return "[{}] {}".format(mode, msg)
    return "\033[{}m[{}] {}\033[0m".format(color, mode, msg)


def is_master() -> bool:
    """Rank-0 check that works with or without an initialised process group."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank() == 0
    except Exception:  # pragma: no cover
        pass
    return int(os.environ.get("RANK", os.environ.get("LOCAL_RANK", "0"))) == 0


def master_print(*args, **kwargs) -> None:
    if is_master():
        print(*args, **kwargs, flush=True)
