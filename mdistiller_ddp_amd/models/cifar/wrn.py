"""Wide ResNets (wrn_16_1/16_2/40_1/40_2), pre-activation blocks.

Layout follows `mdistiller/models/cifar/wrn.py:11-193` (including the fork's
extra ReLU on the stem and between network blocks, `wrn.py:146-152`).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import bn_act, conv_bn_act, pool_linear
from .._base import ModelBase


class BasicBlock(nn.Module):
    def __init__(self, in_planes, out_planes, stride, dropRate=0.0):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(in_planes)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv1 = nn.Conv2d(in_planes, out_planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_planes)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(out_planes, out_planes, 3, 1, 1, bias=False)
        self.droprate = dropRate
        self.equalInOut = in_planes == out_planes
        self.convShortcut = None if self.equalInOut else nn.Conv2d(
            in_planes, out_planes, 1, stride, 0, bias=False)

    def forward(self, x):
        xa, _ = bn_act(x, self.bn1, "relu")
        o, _ = conv_bn_act(xa, self.conv1, self.bn2, "relu", private=self.droprate == 0)
        if self.droprate > 0:
            o = F.dropout(o, p=self.droprate, training=self.training)
        res = x if self.equalInOut else conv_bn_act(xa, self.convShortcut, None, "none")[0]
        return conv_bn_act(o, self.conv2, None, "none", residual=res)[0]


class NetworkBlock(nn.Module):
    def __init__(self, nb_layers, in_planes, out_planes, block, stride, dropRate=0.0):
        super().__init__()
        self.layer = nn.Sequential(*[
            block(in_planes if i == 0 else out_planes, out_planes, stride if i == 0 else 1, dropRate)
            for i in range(nb_layers)])

    def forward(self, x):
        return self.layer(x)


class WideResNet(nn.Module, ModelBase):
    def __init__(self, depth, num_classes, widen_factor=1, dropRate=0.0):
        super().__init__()
        nC = [16, 16 * widen_factor, 32 * widen_factor, 64 * widen_factor]
        assert (depth - 4) % 6 == 0, "depth should be 6n+4"
        n = (depth - 4) // 6
        self.conv1 = nn.Conv2d(3, nC[0], 3, 1, 1, bias=False)
        self.block1 = NetworkBlock(n, nC[0], nC[1], BasicBlock, 1, dropRate)
        self.block2 = NetworkBlock(n, nC[1], nC[2], BasicBlock, 2, dropRate)
        self.block3 = NetworkBlock(n, nC[2], nC[3], BasicBlock, 2, dropRate)
        self.bn1 = nn.BatchNorm2d(nC[3])
        self.relu = nn.ReLU(inplace=True)
        self.fc = nn.Linear(nC[3], num_classes)
        self.nChannels = nC[3]
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                k = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / k))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
            elif isinstance(m, nn.Linear):
                m.bias.data.zero_()
        self.stage_channels = nC

    def get_bn_before_relu(self):
        return [self.block2.layer[0].bn1, self.block3.layer[0].bn1, self.bn1]

    def forward_stem(self, x):
        return conv_bn_act(x, self.conv1, None, "none")[0]

    def get_layers(self):
        return nn.Sequential(self.block1, self.block2, self.block3)

    def forward_pool(self, x):
        out, _ = bn_act(x, self.bn1, "relu")
        out = F.avg_pool2d(out, 8)
        return out.reshape(-1, self.nChannels)

    def get_head(self):
        return self.fc

    def forward(self, x):
        out, f0_pre = conv_bn_act(x, self.conv1, None, "relu", want_preact=True)
        f0 = out
        f1 = self.block1(out)
        f2 = self.block2(F.relu(f1))
        f3 = self.block3(F.relu(f2))
        out, _ = bn_act(f3, self.bn1, "relu")
        avg, logits = pool_linear(out, self.fc, 8)
        return logits, {
            "feats": [f0, F.relu(f1), F.relu(f2), F.relu(f3)],
            "preact_feats": [f0_pre, f1, f2, f3],
            "pooled_feat": avg,
        }


def wrn(**kw):
    return WideResNet(**kw)


def wrn_40_2(**kw):
    return WideResNet(depth=40, widen_factor=2, **kw)


def wrn_40_1(**kw):
    return WideResNet(depth=40, widen_factor=1, **kw)


def wrn_16_2(**kw):
    return WideResNet(depth=16, widen_factor=2, **kw)


def wrn_16_1(**kw):
    return WideResNet(depth=16, widen_factor=1, **kw)
