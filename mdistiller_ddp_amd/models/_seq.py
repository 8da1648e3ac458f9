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


def _defer_to(x, mods, j):
    """"dw" when the group at ``mods[j]`` is a depthwise conv + BN on the
    native training path (ops.hip_train.can_defer_to_depthwise): the group
    before it then leaves its BN apply to that conv's loads."""
    if j >= len(mods) or not isinstance(mods[j], nn.Conv2d):
        return False
    bn = mods[j + 1] if j + 1 < len(mods) and isinstance(mods[j + 1], nn.BatchNorm2d) else None
    from ..ops.nn import hip_enabled_for, _TRAIN_KERNELS
    if bn is None or not hip_enabled_for(x) or not _TRAIN_KERNELS["on"]:
        return False
    from ..ops import hip_layers, hip_train
    if hip_layers.conv_supported(x, mods[j], bn):  # (the inference path would take it)
        return False
    return "dw" if hip_train.can_defer_to_depthwise(x, mods[j], bn) else False


def run_seq(seq, x, residual=None, want_preact=False, final_act=None, next_seq=None):
    """Returns ``(out, preact_of_last_group_or_None)``.

    ``residual`` is added after the last group's BN, before its activation.
    ``final_act`` overrides the last group's activation (e.g. "relu" on a
    linear-bottleneck output whose consumer applies ReLU: one fused launch
    returns both the activated tensor and, with ``want_preact``, the linear
    one).  A conv group followed by a depthwise conv (inside ``seq``, or the
    first group of ``next_seq`` when the caller guarantees that sequence is
    the output's only consumer) hands it its BN + act un-applied
    (ops.hip_train.can_defer_to_depthwise: no apply pass).
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
            defer = False
            if bn is not None and act != "none" and not (last and (want_preact or residual is not None)):
                defer = _defer_to(x, list(next_seq) if last and next_seq is not None else mods,
                                  0 if last else j) if (not last or next_seq is not None) else False
            x, pre = conv_bn_act(x, m, bn, act, residual if last else None, want_preact and last,
                                 defer_apply=defer)
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
