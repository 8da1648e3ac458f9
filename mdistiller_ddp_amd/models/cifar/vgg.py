"""CIFAR VGG-8/11/13/16/19 (BN variants).

Layout follows `mdistiller/models/cifar/vgg.py:28-261`.  ``pool3`` is applied
when the block-3 map is larger than 4x4 -- identical to the reference's
``h == 64`` test for the 32/64-pixel inputs it supports, but also valid in the
staged API where the input size is not visible (`vgg.py:121-122`).
"""
from __future__ import annotations

import math

import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import MaxPool2d, pool_linear
from .._base import ModelBase
from .._seq import run_seq


class _Stage(nn.Module):
    def __init__(self, pool, block, cond_pool=False):
        super().__init__()
        self.pool, self.block, self.cond_pool = pool, block, cond_pool

    def forward(self, x):
        if not self.cond_pool or x.shape[-1] > 4:
            x = self.pool(x)
        return run_seq(self.block, x, want_preact=True)[1]


class VGG(nn.Module, ModelBase):
    def __init__(self, cfg, batch_norm=False, num_classes=1000):
        super().__init__()
        self.block0 = self._make_layers(cfg[0], batch_norm, 3)
        self.block1 = self._make_layers(cfg[1], batch_norm, cfg[0][-1])
        self.block2 = self._make_layers(cfg[2], batch_norm, cfg[1][-1])
        self.block3 = self._make_layers(cfg[3], batch_norm, cfg[2][-1])
        self.block4 = self._make_layers(cfg[4], batch_norm, cfg[3][-1])
        self.pool0 = MaxPool2d(kernel_size=2, stride=2)
        self.pool1 = MaxPool2d(kernel_size=2, stride=2)
        self.pool2 = MaxPool2d(kernel_size=2, stride=2)
        self.pool3 = MaxPool2d(kernel_size=2, stride=2)
        self.pool4 = nn.AdaptiveAvgPool2d((1, 1))
        self.classifier = nn.Linear(512, num_classes)
        self._initialize_weights()
        self.stage_channels = [c[-1] for c in cfg]

    def get_bn_before_relu(self):
        return [self.block1[-1], self.block2[-1], self.block3[-1], self.block4[-1]]

    def forward_stem(self, x):
        return run_seq(self.block0, x, want_preact=True)[1]

    def get_layers(self):
        return nn.Sequential(_Stage(self.pool0, self.block1), _Stage(self.pool1, self.block2),
                             _Stage(self.pool2, self.block3), _Stage(self.pool3, self.block4, True))

    def forward_pool(self, x):
        return self.pool4(F.relu(x)).reshape(x.size(0), -1)

    def get_head(self):
        return self.classifier

    def forward(self, x):
        # each block's last conv applies the ReLU in its own launch and also
        # returns the pre-activation (the stage feature), so no separate ReLU
        # pass runs and the backward stays on the native kernels end to end
        # (DOT's single-pass backward, engine/step.py); the head is the fused
        # pool + classifier (reference models/cifar/vgg.py forward: the same
        # values through F.relu, AdaptiveAvgPool2d and Linear)
        x, f0_pre = run_seq(self.block0, x, want_preact=True, final_act="relu")
        f0 = x
        feats, pres = [f0], [f0_pre]
        for i, (pool, block) in enumerate(((self.pool0, self.block1), (self.pool1, self.block2),
                                            (self.pool2, self.block3), (self.pool3, self.block4))):
            if i < 3 or x.shape[-1] > 4:
                x = pool(x)
            x, pre = run_seq(block, x, want_preact=True, final_act="relu")
            pres.append(pre)
            feats.append(x)
        avg, logits = pool_linear(x, self.classifier)
        return logits, {"feats": feats, "preact_feats": pres, "pooled_feat": avg}

    @staticmethod
    def _make_layers(cfg, batch_norm=False, in_channels=3):
        layers = []
        for v in cfg:
            if v == "M":
                layers += [MaxPool2d(kernel_size=2, stride=2)]
            else:
                conv2d = nn.Conv2d(in_channels, v, kernel_size=3, padding=1)
                layers += [conv2d, nn.BatchNorm2d(v), nn.ReLU(inplace=True)] if batch_norm \
                    else [conv2d, nn.ReLU(inplace=True)]
                in_channels = v
        return nn.Sequential(*layers[:-1])

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


cfg = {
    "A": [[64], [128], [256, 256], [512, 512], [512, 512]],
    "B": [[64, 64], [128, 128], [256, 256], [512, 512], [512, 512]],
    "D": [[64, 64], [128, 128], [256, 256, 256], [512, 512, 512], [512, 512, 512]],
    "E": [[64, 64], [128, 128], [256, 256, 256, 256], [512, 512, 512, 512], [512, 512, 512, 512]],
    "S": [[64], [128], [256], [512], [512]],
}


def vgg8(**kw):
    return VGG(cfg["S"], **kw)


def vgg8_bn(**kw):
    return VGG(cfg["S"], batch_norm=True, **kw)


def vgg11(**kw):
    return VGG(cfg["A"], **kw)


def vgg11_bn(**kw):
    return VGG(cfg["A"], batch_norm=True, **kw)


def vgg13(**kw):
    return VGG(cfg["B"], **kw)


def vgg13_bn(**kw):
    return VGG(cfg["B"], batch_norm=True, **kw)


def vgg16(**kw):
    return VGG(cfg["D"], **kw)


def vgg16_bn(**kw):
    return VGG(cfg["D"], batch_norm=True, **kw)


def vgg19(**kw):
    return VGG(cfg["E"], **kw)


def vgg19_bn(**kw):
    return VGG(cfg["E"], batch_norm=True, **kw)
