"""CIFAR MobileNetV2 (``mobile_half``: T=6, width 0.5).

Layout follows `mdistiller/models/cifar/mobilenetv2.py:26-217` (the stray
``print(T, width_mult)`` of `:117`, SURVEY D19, is dropped).  Pointwise convs
run on the MFMA implicit-GEMM kernel (1x1 = plain GEMM over pixels); the
depthwise 3x3 goes to the dedicated depthwise kernel.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._base import ModelBase
from .._seq import run_seq


def conv_bn(inp, oup, stride):
    return nn.Sequential(nn.Conv2d(inp, oup, 3, stride, 1, bias=False), nn.BatchNorm2d(oup))


def conv_1x1_bn(inp, oup):
    return nn.Sequential(nn.Conv2d(inp, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup),
                         nn.ReLU(inplace=True))


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        assert stride in (1, 2)
        self.blockname = None
        self.stride = stride
        self.use_res_connect = stride == 1 and inp == oup
        hid = inp * expand_ratio
        self.conv = nn.Sequential(
            nn.Conv2d(inp, hid, 1, 1, 0, bias=False), nn.BatchNorm2d(hid), nn.ReLU(inplace=True),
            nn.Conv2d(hid, hid, 3, stride, 1, groups=hid, bias=False), nn.BatchNorm2d(hid),
            nn.ReLU(inplace=True),
            nn.Conv2d(hid, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup),
        )
        self.names = ["0", "1", "2", "3", "4", "5", "6", "7"]

    def forward(self, x):
        return run_seq(self.conv, x, residual=x if self.use_res_connect else None)[0]


class _Group(nn.Module):
    """``blocks[i](relu?(x)) -> blocks[j](...)`` as one staged layer."""

    def __init__(self, *blocks):
        super().__init__()
        self.blocks = blocks

    def forward(self, x):
        for b in self.blocks:
            x = b(x)
        return x


class MobileNetV2(nn.Module, ModelBase):
    def __init__(self, T, feature_dim, input_size=32, width_mult=1.0, remove_avg=False):
        super().__init__()
        self.remove_avg = remove_avg
        self.interverted_residual_setting = [
            [1, 16, 1, 1], [T, 24, 2, 1], [T, 32, 3, 2], [T, 64, 4, 2],
            [T, 96, 3, 1], [T, 160, 3, 2], [T, 320, 1, 1],
        ]
        assert input_size % 32 == 0
        input_channel = int(32 * width_mult)
        self.conv1 = conv_bn(3, input_channel, 2)
        self.blocks = nn.ModuleList([])
        for t, c, n, s in self.interverted_residual_setting:
            output_channel = int(c * width_mult)
            layers = []
            for stride in [s] + [1] * (n - 1):
                layers.append(InvertedResidual(input_channel, output_channel, stride, t))
                input_channel = output_channel
            self.blocks.append(nn.Sequential(*layers))
        self.last_channel = int(1280 * width_mult) if width_mult > 1.0 else 1280
        self.conv2 = conv_1x1_bn(input_channel, self.last_channel)
        self.classifier = nn.Sequential(nn.Linear(self.last_channel, feature_dim))
        self._pool_k = input_size // (32 // 2)
        self.avgpool = nn.AvgPool2d(self._pool_k, ceil_mode=True)
        self._initialize_weights()
        self.stage_channels = [int(c * width_mult) for c in (32, 24, 32, 96, 320)]

    def get_bn_before_relu(self):
        return [self.blocks[1][-1].conv[-1], self.blocks[2][-1].conv[-1],
                self.blocks[4][-1].conv[-1], self.blocks[6][-1].conv[-1]]

    def forward_stem(self, x):
        return run_seq(self.conv1, x)[0]

    def get_layers(self):
        b = self.blocks
        return nn.Sequential(_Group(b[0], b[1]), _Group(b[2]), _Group(b[3], b[4]), _Group(b[5], b[6]))

    def forward_pool(self, x):
        out = run_seq(self.conv2, F.relu(x))[0]
        if not self.remove_avg:
            out = self.avgpool(out)
        return out.reshape(out.size(0), -1)

    def get_head(self):
        return self.classifier

    def forward(self, x):
        out = run_seq(self.conv1, x)[0]
        f0 = out
        out = self.blocks[0](F.relu(out))
        f1 = self.blocks[1](out)
        f2 = self.blocks[2](F.relu(f1))
        out = self.blocks[3](F.relu(f2))
        f3 = self.blocks[4](out)
        out = self.blocks[5](F.relu(f3))
        f4 = self.blocks[6](out)
        out = run_seq(self.conv2, F.relu(f4))[0]
        if not self.remove_avg:
            out = self.avgpool(out)
        avg = out.reshape(out.size(0), -1)
        logits = self.classifier(avg)
        return logits, {
            "feats": [F.relu(f0), F.relu(f1), F.relu(f2), F.relu(f3), F.relu(f4)],
            "preact_feats": [f0, f1, f2, f3, f4],
            "pooled_feat": avg,
        }

    def _initialize_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.weight.data.normal_(0, 0.01)
                m.bias.data.zero_()


def mobilenetv2_T_w(T, W, feature_dim=100):
    return MobileNetV2(T=T, feature_dim=feature_dim, width_mult=W)


def mobile_half(num_classes=100):
    return mobilenetv2_T_w(6, 0.5, num_classes)
