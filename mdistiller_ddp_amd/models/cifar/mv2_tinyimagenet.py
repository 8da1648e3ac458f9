"""Tiny-ImageNet MobileNetV2 (ReLU6, 1x1 stem with padding 1 -> 66x66 maps).

Layout follows `mdistiller/models/cifar/mv2_tinyimagenet.py:7-133`.
``pooled_feat`` is returned flattened to (N, 1280) -- the reference returns the
4-D (N,1280,1,1) tensor, which breaks the pooled-feature distillers (PKT/RKD/
CRD ``torch.mm``); ReviewKD re-adds the spatial dims itself.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import grad_fork, pool_linear
from .._base import ModelBase
from .._seq import run_seq


class LinearBottleNeck(nn.Module):
    def __init__(self, in_channels, out_channels, stride, t=6, class_num=100):
        super().__init__()
        self.residual = nn.Sequential(
            nn.Conv2d(in_channels, in_channels * t, 1), nn.BatchNorm2d(in_channels * t),
            nn.ReLU6(inplace=True),
            nn.Conv2d(in_channels * t, in_channels * t, 3, stride=stride, padding=1,
                      groups=in_channels * t),
            nn.BatchNorm2d(in_channels * t), nn.ReLU6(inplace=True),
            nn.Conv2d(in_channels * t, out_channels, 1), nn.BatchNorm2d(out_channels),
        )
        self.stride, self.in_channels, self.out_channels = stride, in_channels, out_channels

    def forward(self, x, final_act=None):
        """``final_act``: also apply this activation to the block output and
        return ``(activated, linear)`` from the same fused launch."""
        res = x if (self.stride == 1 and self.in_channels == self.out_channels) else None
        # x feeds the expansion conv and the residual add: their input
        # gradients are summed in the native backward (GradFork)
        fork = grad_fork(x) if res is not None else None
        if final_act is None:
            return run_seq(self.residual, x, residual=res, fork=fork)[0]
        return run_seq(self.residual, x, residual=res, want_preact=True, final_act=final_act,
                       fork=fork)


def _stage_act(stage, x):
    """A stage whose output feeds a ReLU6: its last block returns
    (relu6(out), out) from one fused launch."""
    if isinstance(stage, LinearBottleNeck):
        return stage(x, final_act="relu6")
    for blk in list(stage)[:-1]:
        x = blk(x)
    return stage[-1](x, final_act="relu6")


class _Chain(nn.Module):
    def __init__(self, *mods):
        super().__init__()
        self.mods = mods

    def forward(self, x):
        for m in self.mods:
            x = m(x) if not isinstance(m, nn.Sequential) or isinstance(m[0], LinearBottleNeck) \
                else run_seq(m, x)[0]
        return x


class MobileNetV2(nn.Module, ModelBase):
    def __init__(self, num_classes=100):
        super().__init__()
        self.pre = nn.Sequential(nn.Conv2d(3, 32, 1, padding=1), nn.BatchNorm2d(32))
        self.stage1 = LinearBottleNeck(32, 16, 1, 1)
        self.stage2 = self._make_stage(2, 16, 24, 2, 6)
        self.stage3 = self._make_stage(3, 24, 32, 2, 6)
        self.stage4 = self._make_stage(4, 32, 64, 2, 6)
        self.stage5 = self._make_stage(3, 64, 96, 1, 6)
        self.stage6 = self._make_stage(3, 96, 160, 1, 6)
        self.stage7 = LinearBottleNeck(160, 320, 1, 6)
        self.conv1 = nn.Sequential(nn.Conv2d(320, 1280, 1), nn.BatchNorm2d(1280), nn.ReLU6(inplace=True))
        self.conv2 = nn.Conv2d(1280, num_classes, 1)
        self.stage_channels = [32, 24, 32, 64, 1280]

    def activate(self, x):
        return F.relu6(x)

    def forward_stem(self, x):
        return run_seq(self.pre, x)[0]

    def get_layers(self):
        return nn.Sequential(_Chain(self.stage1, self.stage2), _Chain(self.stage3), _Chain(self.stage4),
                             _Chain(self.stage5, self.stage6, self.stage7, self.conv1))

    def forward_pool(self, x):
        return F.adaptive_avg_pool2d(x, 1).flatten(1)

    def get_head(self):
        return _Head(self.conv2)

    def get_bn_before_relu(self):
        return [self.stage2[-1].residual[-1], self.stage3[-1].residual[-1],
                self.stage4[-1].residual[-1], self.conv1[1]]

    def forward(self, x):
        # the reference applies F.relu6 to f0..f3 before their consumers; here
        # each producer emits both tensors from one fused launch, f4 is already
        # ReLU6'd (conv1), and the head is the fused pool + 1x1 classifier --
        # no PyTorch op touches an activation gradient (DOT's single pass)
        a0, f0 = run_seq(self.pre, x, want_preact=True, final_act="relu6")
        x = self.stage1(a0)
        a1, f1 = _stage_act(self.stage2, x)
        a2, f2 = _stage_act(self.stage3, a1)
        a3, f3 = _stage_act(self.stage4, a2)
        x = self.stage5(a3)
        x = self.stage6(x)
        x = self.stage7(x)
        f4 = run_seq(self.conv1, x)[0]
        avg, logits = pool_linear(f4, self.conv2)
        return logits, {
            "feats": [a0, a1, a2, a3, f4],
            "preact_feats": [f0, f1, f2, f3, f4],
            "pooled_feat": avg,
        }

    def _make_stage(self, repeat, in_channels, out_channels, stride, t):
        layers = [LinearBottleNeck(in_channels, out_channels, stride, t)]
        for _ in range(repeat - 1):
            layers.append(LinearBottleNeck(out_channels, out_channels, 1, t))
        return nn.Sequential(*layers)


class _Head(nn.Module):
    def __init__(self, conv):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        return self.conv(x.reshape(x.size(0), -1, 1, 1)).flatten(1)


def mobilenetv2_tinyimagenet(**kw):
    return MobileNetV2(**kw)
