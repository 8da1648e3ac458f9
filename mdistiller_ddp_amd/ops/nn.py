"""Functional layer ops used by every model in the zoo.

Models keep standard ``nn.Conv2d`` / ``nn.BatchNorm2d`` sub-modules (so their
``state_dict`` keys are identical to the reference checkpoints) but run their
forward through these functions.  Each function has two implementations:

* the PyTorch reference (CPU, tests, fallback for shapes the kernels do not
  cover), and
* the HIP path (``ops/hip_layers.py``): one MFMA implicit-GEMM launch per
  conv whose epilogue applies the folded BN affine + residual + activation in
  eval mode, or emits per-channel batch statistics in train mode.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .backend import hip_enabled_for

_ACTS = ("relu", "relu6", "none")
# training-mode native conv+BN path (ops/hip_train.py); switchable for A/B runs
_TRAIN_KERNELS = {"on": True}


def set_train_kernels(flag: bool) -> None:
    _TRAIN_KERNELS["on"] = bool(flag)


def activate(x: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return F.relu(x)
    if act == "relu6":
        return F.relu6(x)
    if act == "none":
        return x
    raise ValueError(act)


def _bn(x: torch.Tensor, bn: nn.BatchNorm2d) -> torch.Tensor:
    return bn(x)


def conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d | None = None,
                act: str = "relu", residual: torch.Tensor | None = None,
                want_preact: bool = False):
    """``act(bn(conv(x)) + residual)``; returns ``(out, preact_or_None)``."""
    if hip_enabled_for(x):
        from . import hip_layers
        if hip_layers.conv_supported(x, conv, bn):
            return hip_layers.conv_bn_act(x, conv, bn, act, residual, want_preact)
        from . import hip_train
        if _TRAIN_KERNELS["on"] and hip_train.train_supported(x, conv, bn):
            return hip_train.conv_bn_act_train(x, conv, bn, act, residual, want_preact)
    y = conv(x)
    if bn is not None:
        y = _bn(y, bn)
    if residual is not None:
        y = y + residual
    out = activate(y, act)
    return out, (y if want_preact else None)


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, act: str = "relu",
           residual: torch.Tensor | None = None, want_preact: bool = False):
    """``act(bn(x) + residual)`` (pre-activation blocks, WRN/ResNet heads)."""
    if hip_enabled_for(x):
        from . import hip_layers
        if hip_layers.bn_supported(x, bn):
            return hip_layers.bn_act(x, bn, act, residual, want_preact)
    y = _bn(x, bn)
    if residual is not None:
        y = y + residual
    out = activate(y, act)
    return out, (y if want_preact else None)


def conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    return conv_bn_act(x, conv, None, "none")[0]


def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.reshape(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


def linear(x: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    return fc(x)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """(N, C, H, W) -> (N, C), fp32-accumulated."""
    return x.float().mean(dim=(2, 3)).to(x.dtype)
