"""Run ``nn.Sequential`` conv chains through the fused conv+BN+act op.

The reference builds VGG / MobileNet blocks as ``nn.Sequential`` lists of
``Conv2d, BatchNorm2d, ReLU`` (so their ``state_dict`` keys are positional,
e.g. ``block0.1.running_mean``).  Keeping those containers preserves checkpoint
compatibility; this helper walks them and groups each ``Conv2d[, BN][, act]``
run into a single fused launch.
"""
from __future__ import annotations

import torch.nn as nn

from ..ops.nn import conv_bn_act, bn_act


def _act_of(m):
    if isinstance(m, nn.ReLU6):
        return "relu6"
    if isinstance(m, nn.ReLU):
        return "relu"
    return None


def run_seq(seq, x, residual=None, want_preact=False, final_act=None, fork=None):
    """Returns ``(out, preact_of_last_group_or_None)``.

    ``residual`` is added after the last group's BN, before its activation.
    ``fork`` (:func:`ops.nn.grad_fork` of ``x`` when ``residual`` is ``x``):
    the first conv and the residual add sum their input gradients inside the
    native backward instead of by an autograd add.
    ``final_act`` overrides the last group's activation (e.g. "relu" on a
    linear-bottleneck output whose consumer applies ReLU: one fused launch
    returns both the activated tensor and, with ``want_preact``, the linear
    one).
    """
    mods = list(seq)
    i, pre = 0, None
    n = len(mods)
    while i < n:
        m = mods[i]
        if isinstance(m, nn.Conv2d):
            bn, act, j = None, "none", i + 1
            if j < n and isinstance(mods[j], nn.BatchNorm2d):
                bn, j = mods[j], j + 1
            if j < n and _act_of(mods[j]) is not None:
                act, j = _act_of(mods[j]), j + 1
            last = j >= n
            if last and final_act is not None:
                act = final_act
            x, pre = conv_bn_act(x, m, bn, act, residual if last else None, want_preact and last,
                                 fork=fork if i == 0 else None,
                                 res_fork=fork if (last and residual is not None) else None)
            i = j
        elif isinstance(m, nn.BatchNorm2d):
            act, j = "none", i + 1
            if j < n and _act_of(mods[j]) is not None:
                act, j = _act_of(mods[j]), j + 1
            last = j >= n
            x, pre = bn_act(x, m, act, residual if last else None, want_preact and last)
            i = j
        else:
            x = m(x)
            pre = x
            i += 1
    return x, pre
