"""CIFAR/Tiny-ImageNet ResNet-18/34/50/101/152 (64-channel 3x3 stem, 4 stages).

Parameter layout follows `mdistiller/models/cifar/resnetv2.py:7-244` (teacher
ResNet50 checkpoints); forward uses the fused-op API.
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import conv_bn_act, pool_linear
from .._base import ModelBase, PreactStage
from .resnet import Stage


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, is_last=False):
        super().__init__()
        self.is_last = is_last
        self._need_preact = True
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes))

    def _res(self, x):
        if len(self.shortcut) == 0:
            return x
        return conv_bn_act(x, self.shortcut[0], self.shortcut[1], "none")[0]

    def forward(self, x):
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", private=True)
        return conv_bn_act(h, self.conv2, self.bn2, "relu", residual=self._res(x),
                           want_preact=self.is_last and self._need_preact)


class Bottleneck(BasicBlock):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, is_last=False):
        nn.Module.__init__(self)
        self.is_last = is_last
        self._need_preact = True
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, self.expansion * planes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(self.expansion * planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes))

    def forward(self, x):
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", private=True)
        h, _ = conv_bn_act(h, self.conv2, self.bn2, "relu", private=True)
        return conv_bn_act(h, self.conv3, self.bn3, "relu", residual=self._res(x),
                           want_preact=self.is_last and self._need_preact)


class ResNet(nn.Module, ModelBase):
    def __init__(self, block, num_blocks, num_classes=10, zero_init_residual=False):
        super().__init__()
        self.in_planes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.linear = nn.Linear(512 * block.expansion, num_classes)
        self._block = block
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)
        e = block.expansion
        self.stage_channels = [64, 64 * e, 128 * e, 256 * e, 512 * e]

    def _make_layer(self, block, planes, num_blocks, stride):
        strides = [stride] + [1] * (num_blocks - 1)
        layers = []
        for i, s in enumerate(strides):
            layers.append(block(self.in_planes, planes, s, i == num_blocks - 1))
            self.in_planes = planes * block.expansion
        return Stage(*layers)

    def get_bn_before_relu(self):
        last = "bn3" if self._block is Bottleneck else "bn2"
        return [getattr(l[-1], last) for l in (self.layer1, self.layer2, self.layer3, self.layer4)]

    def encode(self, x, idx, preact=False):
        """Run one late stage on a pre-activation input (reference `resnetv2.py:160-169`)."""
        layer = {-1: self.layer4, -2: self.layer3, -3: self.layer2}.get(idx)
        if layer is None:
            raise NotImplementedError(idx)
        out, pre = layer(F.relu(x))
        return pre

    def forward_stem(self, x):
        return self.bn1(self.conv1(x))

    def get_layers(self):
        return nn.Sequential(*[PreactStage(l) for l in (self.layer1, self.layer2, self.layer3, self.layer4)])

    def forward_pool(self, x):
        return self.avgpool(F.relu(x)).reshape(x.size(0), -1)

    def get_head(self):
        return self.linear

    def forward(self, x):
        need = self._need_preact
        out, f0_pre = conv_bn_act(x, self.conv1, self.bn1, "relu", want_preact=need)
        f0 = out
        out, f1_pre = self.layer1(out)
        f1 = out
        out, f2_pre = self.layer2(out)
        f2 = out
        out, f3_pre = self.layer3(out)
        f3 = out
        out, f4_pre = self.layer4(out)
        f4 = out
        avg, logits = pool_linear(out, self.linear)  # fused pool + classifier
        return logits, {
            "feats": [f0, f1, f2, f3, f4],
            "preact_feats": [f0_pre, f1_pre, f2_pre, f3_pre, f4_pre],
            "pooled_feat": avg,
        }


def ResNet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def ResNet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def ResNet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def ResNet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


def ResNet152(**kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], **kw)
