"""ImageNet MobileNetV1 (student of the R50->MV1 configs).

Layout follows `mdistiller/models/imagenet/mobilenetv1.py:8-97`
(``model.{0..14}``, ``fc``); stage ends are the ``act=False`` depthwise-separable
blocks.  Depthwise 3x3 convs run on the dedicated HIP stencil kernel, the
pointwise 1x1 convs on the MFMA implicit-GEMM kernel.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import pool_linear

from .._base import ModelBase
from .._seq import run_seq


def _conv_bn(inp, oup, stride):
    return nn.Sequential(nn.Conv2d(inp, oup, 3, stride, 1, bias=False), nn.BatchNorm2d(oup),
                         nn.ReLU(inplace=True))


def _conv_dw(inp, oup, stride, act=True):
    layers = [nn.Conv2d(inp, inp, 3, stride, 1, groups=inp, bias=False), nn.BatchNorm2d(inp),
              nn.ReLU(inplace=True), nn.Conv2d(inp, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup)]
    if act:
        layers.append(nn.ReLU(inplace=True))
    return nn.Sequential(*layers)


class _Range(nn.Module):
    def __init__(self, mods):
        super().__init__()
        self.mods = tuple(mods)

    def forward(self, x):
        for m in self.mods:
            x = run_seq(m, x)[0]
        return x


class MobileNetV1(nn.Module, ModelBase):
    STAGES = ((1, 3), (3, 5), (5, 11), (11, 14))

    def __init__(self, num_classes=1000, **kwargs):
        super().__init__()
        self.model = nn.Sequential(
            _conv_bn(3, 32, 2), _conv_dw(32, 64, 1), _conv_dw(64, 128, 2, act=False),
            _conv_dw(128, 128, 1), _conv_dw(128, 256, 2, act=False),
            _conv_dw(256, 256, 1), _conv_dw(256, 512, 2), _conv_dw(512, 512, 1),
            _conv_dw(512, 512, 1), _conv_dw(512, 512, 1), _conv_dw(512, 512, 1, act=False),
            _conv_dw(512, 512, 1), _conv_dw(512, 1024, 2), _conv_dw(1024, 1024, 1, act=False),
            nn.AvgPool2d(7),
        )
        self.fc = nn.Linear(1024, num_classes)
        self.stage_channels = [32, 128, 256, 512, 1024]

    def forward_stem(self, x):
        return run_seq(self.model[0], x, want_preact=True)[1]

    def get_layers(self):
        return nn.Sequential(*[_Range(self.model[a:b]) for a, b in self.STAGES])

    def forward_pool(self, x):
        return F.adaptive_avg_pool2d(F.relu(x), 1).reshape(x.size(0), -1)

    def get_head(self):
        return self.fc

    def forward(self, x, is_feat=False):
        stem, stem_pre = run_seq(self.model[0], x, want_preact=True)
        feats, pres = [stem], [stem_pre]
        h = stem
        for a, b in self.STAGES:
            for i in range(a, b):
                h = run_seq(self.model[i], h)[0]
            pres.append(h)
            h = F.relu(h)
            feats.append(h)
        avg, logits = pool_linear(h, self.fc)
        return logits, {"pooled_feat": avg, "feats": feats, "preact_feats": pres}

    def get_bn_before_relu(self):
        return [self.model[2][4], self.model[4][4], self.model[10][4], self.model[13][4]]
