"""Tiny-ImageNet MobileNetV2 (ReLU6, 1x1 stem with padding 1 -> 66x66 maps).

Layout follows `mdistiller/models/cifar/mv2_tinyimagenet.py:7-133`.
``pooled_feat`` is returned flattened to (N, 1280) -- the reference returns the
4-D (N,1280,1,1) tensor, which breaks the pooled-feature distillers (PKT/RKD/
CRD ``torch.mm``); ReviewKD re-adds the spatial dims itself.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

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

    def forward(self, x):
        res = x if (self.stride == 1 and self.in_channels == self.out_channels) else None
        return run_seq(self.residual, x, residual=res)[0]


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
        f0 = run_seq(self.pre, x)[0]
        x = self.stage1(F.relu6(f0))
        f1 = self.stage2(x)
        f2 = self.stage3(F.relu6(f1))
        f3 = self.stage4(F.relu6(f2))
        x = self.stage5(F.relu6(f3))
        x = self.stage6(x)
        x = self.stage7(x)
        f4 = run_seq(self.conv1, x)[0]
        avg = F.adaptive_avg_pool2d(f4, 1)
        logits = self.conv2(avg).flatten(1)
        return logits, {
            "feats": [F.relu6(f0), F.relu6(f1), F.relu6(f2), F.relu6(f3), F.relu6(f4)],
            "preact_feats": [f0, f1, f2, f3, f4],
            "pooled_feat": avg.flatten(1),
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
