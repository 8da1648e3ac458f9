"""Kernel-backend selection.

Two backends implement every op in :mod:`mdistiller_ddp_amd.ops`:

* ``"torch"`` -- plain PyTorch ops.  The numerical reference for every HIP
  kernel, and the CPU path (tests, the CPU plumbing config).
* ``"hip"``   -- hand-written CDNA4 kernels from ``ops/csrc`` (MFMA implicit-GEMM
  convolutions with fused BN/activation epilogues, fused losses, fused
  optimizers).  Used for CUDA tensors when the extension is built.

``"auto"`` resolves to ``hip`` whenever a GPU is visible.  On a GPU box the
HIP extension is REQUIRED in auto mode: a missing/broken build raises instead
of silently running the PyTorch path (the round-end checks record which
native objects were actually loaded).
"""
from __future__ import annotations

import os
import threading

_state = threading.local()
_GLOBAL = {"backend": os.environ.get("MDA_BACKEND", "auto")}


def set_backend(name: str) -> None:
    if name not in ("auto", "hip", "torch"):
        raise ValueError(f"unknown backend {name!r}")
    _GLOBAL["backend"] = name


def requested_backend() -> str:
    return getattr(_state, "override", None) or _GLOBAL["backend"]


class use_backend:
    """Context manager: temporarily force a backend (thread-local)."""

    def __init__(self, name: str):
        self.name = name
        self.prev = None

    def __enter__(self):
        self.prev = getattr(_state, "override", None)
        _state.override = self.name
        return self

    def __exit__(self, *exc):
        _state.override = self.prev
        return False


def hip_enabled_for(t) -> bool:
    """True when op inputs living on ``t``'s device should take the HIP path."""
    be = requested_backend()
    if be == "torch" or not getattr(t, "is_cuda", False):
        return False
    from . import _ext
    if be == "hip":
        _ext.load(required=True)
        return True
    # auto
    return _ext.load(required=_ext.gpu_box()) is not None
