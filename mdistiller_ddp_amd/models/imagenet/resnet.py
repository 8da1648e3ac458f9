"""ImageNet ResNet-18/34/50/101/152 (torchvision parameter layout).

Follows `mdistiller/models/imagenet/resnet.py:29-273`: blocks hand over the
pre-ReLU sum and the next block applies the ReLU, so stage outputs are
pre-activations.  In the fused form the ReLU is produced by the same kernel
that produces the pre-activation (one launch, two outputs when the preact is
consumed).  ``pretrained=True`` loads a local torchvision-format checkpoint
(``$MDA_PRETRAINED_DIR/resnetXX.pth``); there is no network download.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import MaxPool2d, conv_bn_act, grad_fork, pool_linear
from ...ops.hip_train import arm_apply_ride, can_defer_residual, finish_apply_ride
from ...runtime.streams import run_branch
from .._base import ModelBase, PreactStage
from ..cifar.resnet import Stage


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride
        self.is_last = False
        self._need_preact = True

    def _res(self, x, fork=None, h=None, conv=None, bn=None):
        """(residual, residual fork): the projection shortcut runs on the
        branch stream; x's two consumers sum their gradients in the native
        backward (ops.hip_train.GradFork).  Its BN is applied inside the
        consumer's (``conv``/``bn`` on ``h``) apply when that one is native
        (ops.hip_train.VirtualBN)."""
        if self.downsample is None:
            return x, fork
        defer = conv is not None and can_defer_residual(h, conv, bn)
        fn = (lambda t: conv_bn_act(t, self.downsample[0], self.downsample[1],
                                    "none", fork=fork, defer_apply=defer)[0])
        res = run_branch(x, fn)
        return res, None

    def forward(self, x):
        fork = grad_fork(x)
        if self.downsample is not None:
            arm_apply_ride(x)  # conv1's BN apply rides in the shortcut's launch
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", fork=fork, private=True)
        res, res_fork = self._res(x, fork, h, self.conv2, self.bn2)  # after conv1: its backward runs first
        finish_apply_ride()
        return conv_bn_act(h, self.conv2, self.bn2, "relu", residual=res,
                           want_preact=self.is_last and self._need_preact, res_fork=res_fork,
                           private=not (self.is_last and self._need_preact))


class Bottleneck(BasicBlock):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        nn.Module.__init__(self)
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.is_last = False
        self._need_preact = True

    def forward(self, x):
        fork = grad_fork(x)
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", fork=fork, private=True)
        h, _ = conv_bn_act(h, self.conv2, self.bn2, "relu", private=True)
        res, res_fork = self._res(x, fork, h, self.conv3, self.bn3)  # after conv1: its backward runs first
        return conv_bn_act(h, self.conv3, self.bn3, "relu", residual=res,
                           want_preact=self.is_last and self._need_preact, res_fork=res_fork,
                           private=not (self.is_last and self._need_preact))


class ResNet(nn.Module, ModelBase):
    def __init__(self, block, layers, num_classes=1000):
        self.inplanes = 64
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AvgPool2d(7, stride=1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        self._block = block
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        e = block.expansion
        self.stage_channels = [64, 64 * e, 128 * e, 256 * e, 512 * e]

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        layers[-1].is_last = True
        return Stage(*layers)

    def get_bn_before_relu(self):
        # last three stages, as the reference (`imagenet/resnet.py:149-166`);
        # OFD aligns its connector list to this length.
        last = "bn3" if self._block is Bottleneck else "bn2"
        return [getattr(l[-1], last) for l in (self.layer2, self.layer3, self.layer4)]

    def forward_stem(self, x):
        x = self.bn1(self.conv1(x))
        return self.maxpool(x)

    def get_layers(self):
        return nn.Sequential(*[PreactStage(l) for l in (self.layer1, self.layer2, self.layer3, self.layer4)])

    def forward_pool(self, x):
        x = F.adaptive_avg_pool2d(F.relu(x), 1)
        return x.view(x.size(0), -1)

    def get_head(self):
        return self.fc

    def forward(self, x):
        need = self._need_preact
        x, stem_pre = conv_bn_act(x, self.conv1, self.bn1, "relu", want_preact=need)
        x = self.maxpool(x)
        f0 = x
        f0_pre = self.maxpool(stem_pre) if stem_pre is not None else None
        x, p1 = self.layer1(x)
        f1 = x
        x, p2 = self.layer2(x)
        f2 = x
        x, p3 = self.layer3(x)
        f3 = x
        x, p4 = self.layer4(x)
        f4 = x
        avg, out = pool_linear(x, self.fc)
        return out, {"pooled_feat": avg, "feats": [f0, f1, f2, f3, f4],
                     "preact_feats": [f0_pre, p1, p2, p3, p4]}


def _load_pretrained(model, name):
    root = os.environ.get("MDA_PRETRAINED_DIR", "")
    path = os.path.join(root, f"{name}.pth")
    if not root or not os.path.exists(path):
        raise FileNotFoundError(
            f"pretrained weights for {name} not found ({path!r}); set MDA_PRETRAINED_DIR to a directory "
            f"holding torchvision-format '{name}.pth' files (no network access is used)")
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd.get("model", sd) if isinstance(sd, dict) else sd)
    return model


def resnet18(pretrained=False, **kw):
    m = ResNet(BasicBlock, [2, 2, 2, 2], **kw)
    return _load_pretrained(m, "resnet18") if pretrained else m


def resnet34(pretrained=False, **kw):
    m = ResNet(BasicBlock, [3, 4, 6, 3], **kw)
    return _load_pretrained(m, "resnet34") if pretrained else m


def resnet50(pretrained=False, **kw):
    m = ResNet(Bottleneck, [3, 4, 6, 3], **kw)
    return _load_pretrained(m, "resnet50") if pretrained else m


def resnet101(pretrained=False, **kw):
    m = ResNet(Bottleneck, [3, 4, 23, 3], **kw)
    return _load_pretrained(m, "resnet101") if pretrained else m


def resnet152(pretrained=False, **kw):
    m = ResNet(Bottleneck, [3, 8, 36, 3], **kw)
    return _load_pretrained(m, "resnet152") if pretrained else m
