"""CIFAR ResNets (resnet8 ... resnet110, resnet8x4, resnet32x4).

Architecture and ``state_dict`` layout follow the reference
(`mdistiller/models/cifar/resnet.py:17-274`) so its teacher checkpoints load
unchanged; the forward is written against the fused-op API
(:func:`ops.nn.conv_bn_act`), so on MI355X each conv+BN(+residual)+ReLU is one
MFMA implicit-GEMM launch, and the block contract is "activated input ->
(activated output, pre-activation)".
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import conv_bn_act, grad_fork, pool_linear
from ...ops.hip_train import arm_apply_ride, can_defer_residual, finish_apply_ride
from ...runtime.streams import run_branch
from .._base import ModelBase, PreactStage


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, is_last=False):
        super().__init__()
        self.is_last = is_last
        self._need_preact = True
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def _shortcut(self, x, fork=None, defer=False):
        return conv_bn_act(x, self.downsample[0], self.downsample[1], "none", fork=fork,
                           defer_apply=defer)[0]

    def forward(self, x):
        # x feeds conv1 and the shortcut: their input gradients are summed in
        # the second one's dgrad epilogue (GradFork), not by an autograd add
        fork = grad_fork(x)
        if self.downsample is not None:
            # conv1's BN apply rides in the projection shortcut's conv launch
            # (ops/hip_train.py arm_apply_ride); nothing reads h before it
            arm_apply_ride(x)
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", fork=fork, private=True)
        if self.downsample is None:
            res = x
        else:
            # projection shortcut (on the branch stream), beside
            # conv2.  Created after conv1, so autograd issues its backward
            # first: the shorter branch chain (BN backward + 1x1 dgrad) parks
            # its input gradient and conv1's dgrad, last on the main chain, adds
            # it in its epilogue.  Its BN is applied inside bn2's apply
            # (ops/hip_train.py VirtualBN)
            defer = can_defer_residual(h, self.conv2, self.bn2)
            res = run_branch(x, lambda t: self._shortcut(t, fork, defer))
            finish_apply_ride()
            fork = None
        # the block output is a stage feature only when features are consumed
        return conv_bn_act(h, self.conv2, self.bn2, "relu", residual=res,
                           want_preact=self.is_last and self._need_preact, res_fork=fork,
                           private=not (self.is_last and self._need_preact))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, is_last=False):
        super().__init__()
        self.is_last = is_last
        self._need_preact = True
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def _shortcut(self, x, fork=None, defer=False):
        return conv_bn_act(x, self.downsample[0], self.downsample[1], "none", fork=fork,
                           defer_apply=defer)[0]

    def forward(self, x):
        fork = grad_fork(x)
        h, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", fork=fork, private=True)
        h, _ = conv_bn_act(h, self.conv2, self.bn2, "relu", private=True)
        res = x if self.downsample is None else run_branch(
            x, lambda t: self._shortcut(t, fork, can_defer_residual(h, self.conv3, self.bn3)))
        return conv_bn_act(h, self.conv3, self.bn3, "relu", residual=res,
                           want_preact=self.is_last and self._need_preact,
                           res_fork=fork if self.downsample is None else None,
                           private=not (self.is_last and self._need_preact))


class Stage(nn.Sequential):
    """A run of blocks: activated input -> (activated output, last preact)."""

    def forward(self, x):
        pre = None
        for blk in self:
            x, pre = blk(x)
        return x, pre


class ResNet(nn.Module, ModelBase):
    def __init__(self, depth, num_filters, block_name="BasicBlock", num_classes=10):
        super().__init__()
        if block_name.lower() == "basicblock":
            assert (depth - 2) % 6 == 0, "basicblock depth must be 6n+2"
            n, block = (depth - 2) // 6, BasicBlock
        elif block_name.lower() == "bottleneck":
            assert (depth - 2) % 9 == 0, "bottleneck depth must be 9n+2"
            n, block = (depth - 2) // 9, Bottleneck
        else:
            raise ValueError("block_name should be BasicBlock or Bottleneck")
        self.inplanes = num_filters[0]
        self.conv1 = nn.Conv2d(3, num_filters[0], kernel_size=3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(num_filters[0])
        self.relu = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(block, num_filters[1], n)
        self.layer2 = self._make_layer(block, num_filters[2], n, stride=2)
        self.layer3 = self._make_layer(block, num_filters[3], n, stride=2)
        self.avgpool = nn.AvgPool2d(8)
        self.fc = nn.Linear(num_filters[3] * block.expansion, num_classes)
        self.stage_channels = list(num_filters)
        self._block = block
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1,
                          stride=stride, bias=False),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample, is_last=(blocks == 1))]
        self.inplanes = planes * block.expansion
        for i in range(1, blocks):
            layers.append(block(self.inplanes, planes, is_last=(i == blocks - 1)))
        return Stage(*layers)

    # contract helpers -----------------------------------------------------
    def get_bn_before_relu(self):
        last = "bn3" if self._block is Bottleneck else "bn2"
        return [getattr(self.layer1[-1], last), getattr(self.layer2[-1], last),
                getattr(self.layer3[-1], last)]

    def forward_stem(self, x):
        return self.bn1(self.conv1(x))

    def get_layers(self):
        return nn.Sequential(PreactStage(self.layer1), PreactStage(self.layer2),
                             PreactStage(self.layer3))

    def forward_pool(self, x):
        x = F.avg_pool2d(F.relu(x), 8)
        return x.reshape(x.size(0), -1)

    def get_head(self):
        return self.fc

    def forward(self, x):
        need = self._need_preact
        # logit-only consumers (need False): no feature takes a gradient, so
        # the stage outputs are private to the native layers (BnLink.private)
        x, f0_pre = conv_bn_act(x, self.conv1, self.bn1, "relu", want_preact=need, private=not need)
        f0 = x
        x, f1_pre = self.layer1(x)
        f1 = x
        x, f2_pre = self.layer2(x)
        f2 = x
        x, f3_pre = self.layer3(x)
        f3 = x
        avg, out = pool_linear(x, self.fc, 8)
        return out, {
            "feats": [f0, f1, f2, f3],
            "preact_feats": [f0_pre, f1_pre, f2_pre, f3_pre],
            "pooled_feat": avg,
        }


def resnet8(**kw):
    return ResNet(8, [16, 16, 32, 64], "basicblock", **kw)


def resnet14(**kw):
    return ResNet(14, [16, 16, 32, 64], "basicblock", **kw)


def resnet20(**kw):
    return ResNet(20, [16, 16, 32, 64], "basicblock", **kw)


def resnet32(**kw):
    return ResNet(32, [16, 16, 32, 64], "basicblock", **kw)


def resnet44(**kw):
    return ResNet(44, [16, 16, 32, 64], "basicblock", **kw)


def resnet56(**kw):
    return ResNet(56, [16, 16, 32, 64], "basicblock", **kw)


def resnet110(**kw):
    return ResNet(110, [16, 16, 32, 64], "basicblock", **kw)


def resnet8x4(**kw):
    return ResNet(8, [32, 64, 128, 256], "basicblock", **kw)


def resnet32x4(**kw):
    return ResNet(32, [32, 64, 128, 256], "basicblock", **kw)
