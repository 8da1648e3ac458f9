"""Detection backbones: ResNet-18/34/50/101/152 (the reference adds BasicBlock
and depth 18 to Detectron2's ResNet, `detection/model/backbone/resnet.py:52-117,
472-550`), MobileNetV2 (`backbone/mobilenetv2.py:63-213`) and FPN with the P6
max-pool top block (`backbone/fpn.py:9-52`).  Parameter names follow
Detectron2's layout (``res2.0.conv1.weight``, ``conv1.norm.*``,
``fpn_lateral2``, ``bottom_up.features.N.conv.M``) so its checkpoints load.

Every conv + BN/FrozenBN (+ residual) (+ ReLU/ReLU6) goes through the fused
op (:func:`..ops.nn.conv_bn_act`): for the frozen teacher and frozen student
stages that is ONE MFMA implicit-GEMM launch with the BN folded into the
packed weights (``ops/hip_layers.py``), and the FPN's lateral 1x1 conv adds
the upsampled top-down map in its epilogue (the residual operand).
Deformable-conv stages (``RESNETS.DEFORM_ON_PER_STAGE``) are not built:
no reference config enables them.
"""
from __future__ import annotations

import math
from collections import namedtuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models._seq import run_seq
from ..ops.nn import activate, conv_bn_act

ShapeSpec = namedtuple("ShapeSpec", ["channels", "stride"])


class FrozenBatchNorm2d(nn.BatchNorm2d):
    """BatchNorm whose statistics and affine are fixed (always in eval mode).

    A ``BatchNorm2d`` subclass, so the fused conv path folds it like any
    eval-mode BN; its affine parameters have ``requires_grad=False``.
    """

    def __init__(self, num_features, eps=1e-5):
        super().__init__(num_features, eps=eps)
        self.weight.requires_grad_(False)
        self.bias.requires_grad_(False)
        nn.Module.train(self, False)

    def train(self, mode=True):
        return self

    @classmethod
    def convert_frozen_batchnorm(cls, module):
        if isinstance(module, nn.BatchNorm2d) and not isinstance(module, cls):
            res = cls(module.num_features, module.eps)
            with torch.no_grad():
                if module.affine:
                    res.weight.copy_(module.weight)
                    res.bias.copy_(module.bias)
                res.running_mean.copy_(module.running_mean)
                res.running_var.copy_(module.running_var)
            return res.to(module.running_mean.device)
        for name, child in module.named_children():
            new = cls.convert_frozen_batchnorm(child)
            if new is not child:
                setattr(module, name, new)
        return module


def get_norm(norm, out_channels):
    if norm in (None, ""):
        return None
    if not isinstance(norm, str):
        return norm(out_channels)
    return {"BN": nn.BatchNorm2d, "SyncBN": nn.BatchNorm2d, "nnSyncBN": nn.BatchNorm2d,
            "FrozenBN": FrozenBatchNorm2d,
            "GN": lambda c: nn.GroupNorm(32, c)}[norm](out_channels)


def c2_msra_fill(m: nn.Module) -> None:
    nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
    if m.bias is not None:
        nn.init.constant_(m.bias, 0)


def c2_xavier_fill(m: nn.Module) -> None:
    nn.init.kaiming_uniform_(m.weight, a=1)
    if m.bias is not None:
        nn.init.constant_(m.bias, 0)


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` with an optional ``norm`` child and activation
    (Detectron2's layout); ``forward(x, residual)`` = act(norm(conv(x)) + residual)."""

    def __init__(self, *args, norm=None, activation=None, **kwargs):
        super().__init__(*args, **kwargs)
        self.norm = norm
        self.activation = activation

    def forward(self, x, residual=None):
        act = self.activation or "none"
        if self.norm is None or isinstance(self.norm, nn.BatchNorm2d):
            return conv_bn_act(x, self, self.norm, act, residual)[0]
        y = self.norm(self._conv_forward(x, self.weight, self.bias))
        if residual is not None:
            y = y + residual
        return activate(y, act)


class _Block(nn.Module):
    def freeze(self):
        for p in self.parameters():
            p.requires_grad = False
        FrozenBatchNorm2d.convert_frozen_batchnorm(self)
        return self


# ----------------------------------------------------------------------------- ResNet
class BasicStem(_Block):
    def __init__(self, in_channels=3, out_channels=64, norm="BN"):
        super().__init__()
        self.conv1 = Conv2d(in_channels, out_channels, kernel_size=7, stride=2, padding=3, bias=False,
                            norm=get_norm(norm, out_channels), activation="relu")
        c2_msra_fill(self.conv1)
        self.out_channels = out_channels
        self.stride = 4

    def forward(self, x):
        return F.max_pool2d(self.conv1(x), kernel_size=3, stride=2, padding=1)


class BasicBlock(_Block):
    def __init__(self, in_channels, out_channels, *, bottleneck_channels=None, stride=1, num_groups=1,
                 norm="BN", stride_in_1x1=False, dilation=1):
        super().__init__()
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride
        self.shortcut = (Conv2d(in_channels, out_channels, 1, stride=stride, bias=False,
                                norm=get_norm(norm, out_channels))
                         if in_channels != out_channels else None)
        self.conv1 = Conv2d(in_channels, out_channels, 3, stride=stride, padding=dilation, bias=False,
                            groups=num_groups, dilation=dilation, norm=get_norm(norm, out_channels),
                            activation="relu")
        self.conv2 = Conv2d(out_channels, out_channels, 3, stride=1, padding=1, bias=False,
                            groups=num_groups, norm=get_norm(norm, out_channels), activation="relu")
        for layer in (self.conv1, self.conv2, self.shortcut):
            if layer is not None:
                c2_msra_fill(layer)

    def forward(self, x):
        sc = self.shortcut(x) if self.shortcut is not None else x
        return self.conv2(self.conv1(x), residual=sc)


class BottleneckBlock(_Block):
    def __init__(self, in_channels, out_channels, *, bottleneck_channels, stride=1, num_groups=1,
                 norm="BN", stride_in_1x1=False, dilation=1):
        super().__init__()
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride
        self.shortcut = (Conv2d(in_channels, out_channels, 1, stride=stride, bias=False,
                                norm=get_norm(norm, out_channels))
                         if in_channels != out_channels else None)
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = Conv2d(in_channels, bottleneck_channels, 1, stride=s1, bias=False,
                            norm=get_norm(norm, bottleneck_channels), activation="relu")
        self.conv2 = Conv2d(bottleneck_channels, bottleneck_channels, 3, stride=s3, padding=dilation,
                            bias=False, groups=num_groups, dilation=dilation,
                            norm=get_norm(norm, bottleneck_channels), activation="relu")
        self.conv3 = Conv2d(bottleneck_channels, out_channels, 1, bias=False,
                            norm=get_norm(norm, out_channels), activation="relu")
        for layer in (self.conv1, self.conv2, self.conv3, self.shortcut):
            if layer is not None:
                c2_msra_fill(layer)

    def forward(self, x):
        sc = self.shortcut(x) if self.shortcut is not None else x
        return self.conv3(self.conv2(self.conv1(x)), residual=sc)


class DeformBottleneckBlock(_Block):
    """Bottleneck with a deformable 3x3 (reference ``backbone/resnet.py:223-336``):
    a plain 3x3 conv predicts per-tap offsets (and, modulated, a sigmoid mask)
    from the 1x1 output; it starts at zero so the block begins as a regular
    bottleneck."""

    def __init__(self, in_channels, out_channels, *, bottleneck_channels, stride=1, num_groups=1,
                 norm="BN", stride_in_1x1=False, dilation=1, deform_modulated=False,
                 deform_num_groups=1):
        super().__init__()
        from .deform import DeformConv, ModulatedDeformConv
        self.in_channels, self.out_channels, self.stride = in_channels, out_channels, stride
        self.deform_modulated = deform_modulated
        self.shortcut = (Conv2d(in_channels, out_channels, 1, stride=stride, bias=False,
                                norm=get_norm(norm, out_channels))
                         if in_channels != out_channels else None)
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = Conv2d(in_channels, bottleneck_channels, 1, stride=s1, bias=False,
                            norm=get_norm(norm, bottleneck_channels), activation="relu")
        per_group = 27 if deform_modulated else 18  # (2 offsets [+ 1 mask]) x 3 x 3 taps
        self.conv2_offset = Conv2d(bottleneck_channels, per_group * deform_num_groups, 3, stride=s3,
                                   padding=dilation, dilation=dilation)
        op = ModulatedDeformConv if deform_modulated else DeformConv
        self.conv2 = op(bottleneck_channels, bottleneck_channels, 3, stride=s3, padding=dilation,
                        bias=False, groups=num_groups, dilation=dilation,
                        deformable_groups=deform_num_groups, norm=get_norm(norm, bottleneck_channels))
        self.conv3 = Conv2d(bottleneck_channels, out_channels, 1, bias=False,
                            norm=get_norm(norm, out_channels), activation="relu")
        for layer in (self.conv1, self.conv2, self.conv3, self.shortcut):
            if layer is not None:
                c2_msra_fill(layer)
        nn.init.constant_(self.conv2_offset.weight, 0)
        nn.init.constant_(self.conv2_offset.bias, 0)

    def forward(self, x):
        out = self.conv1(x)
        if self.deform_modulated:
            om = self.conv2_offset(out)
            n = om.shape[1] // 3
            out = self.conv2(out, om[:, : 2 * n], om[:, 2 * n:].sigmoid())
        else:
            out = self.conv2(out, self.conv2_offset(out))
        out = F.relu(out)
        sc = self.shortcut(x) if self.shortcut is not None else x
        return self.conv3(out, residual=sc)


class ResNet(nn.Module):
    def __init__(self, stem, stages, out_features):
        super().__init__()
        self.stem = stem
        stride = stem.stride
        self._out_feature_strides = {"stem": stride}
        self._out_feature_channels = {"stem": stem.out_channels}
        self.stage_names = []
        for i, blocks in enumerate(stages):
            name = f"res{i + 2}"
            self.add_module(name, nn.Sequential(*blocks))
            self.stage_names.append(name)
            for b in blocks:
                stride *= b.stride
            self._out_feature_strides[name] = stride
            self._out_feature_channels[name] = blocks[-1].out_channels
        self._out_features = list(out_features)

    def forward(self, x):
        out = {}
        x = self.stem(x)
        if "stem" in self._out_features:
            out["stem"] = x
        for name in self.stage_names:
            x = getattr(self, name)(x)
            if name in self._out_features:
                out[name] = x
        return out

    def output_shape(self):
        return {n: ShapeSpec(self._out_feature_channels[n], self._out_feature_strides[n])
                for n in self._out_features}


_BLOCKS_PER_DEPTH = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3],
                     152: [3, 8, 36, 3]}


def build_resnet_backbone(mcfg, in_channels: int = 3) -> ResNet:
    """``mcfg`` = ``cfg.MODEL`` (or ``cfg.TEACHER.MODEL``)."""
    r = mcfg.RESNETS
    norm = r.NORM
    stem = BasicStem(in_channels, r.STEM_OUT_CHANNELS, norm)
    freeze_at = mcfg.BACKBONE.FREEZE_AT
    if freeze_at >= 1:
        stem.freeze()
    depth = r.DEPTH
    out_features = list(r.OUT_FEATURES)
    bott = r.NUM_GROUPS * r.WIDTH_PER_GROUP
    in_ch, out_ch = r.STEM_OUT_CHANNELS, r.RES2_OUT_CHANNELS
    if depth in (18, 34):
        assert out_ch == 64, "R18/R34 need MODEL.RESNETS.RES2_OUT_CHANNELS = 64"
        assert r.RES5_DILATION == 1, "R18/R34 do not support dilation in res5"
    max_stage = max({"res2": 2, "res3": 3, "res4": 4, "res5": 5}.get(f, 2) for f in out_features)
    cls = BasicBlock if depth < 50 else BottleneckBlock
    stages = []
    for idx, stage_idx in enumerate(range(2, max_stage + 1)):
        dil = r.RES5_DILATION if stage_idx == 5 else 1
        first_stride = 1 if idx == 0 or (stage_idx == 5 and dil == 2) else 2
        blocks = []
        deform = bool(r.DEFORM_ON_PER_STAGE[idx])
        if deform and depth < 50:
            raise ValueError("deformable stages need bottleneck blocks (ResNet-50 and deeper)")
        for i in range(_BLOCKS_PER_DEPTH[depth][idx]):
            kw = dict(bottleneck_channels=bott, stride=first_stride if i == 0 else 1,
                      num_groups=r.NUM_GROUPS, norm=norm, stride_in_1x1=r.STRIDE_IN_1X1, dilation=dil)
            if deform:
                blocks.append(DeformBottleneckBlock(in_ch, out_ch, deform_modulated=r.DEFORM_MODULATED,
                                                    deform_num_groups=r.DEFORM_NUM_GROUPS, **kw))
            else:
                blocks.append(cls(in_ch, out_ch, **kw))
            in_ch = out_ch
        out_ch *= 2
        bott *= 2
        if freeze_at >= stage_idx:
            for b in blocks:
                b.freeze()
        stages.append(blocks)
    return ResNet(stem, stages, out_features)


# ----------------------------------------------------------------------------- MobileNetV2
def _make_divisible(v, divisor, min_value=None):
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def _norm_or_identity(norm, c):
    n = get_norm(norm, c)
    return nn.Identity() if n is None else n


class InvertedResidual(_Block):
    def __init__(self, inp, oup, stride, expand_ratio, norm):
        super().__init__()
        assert stride in (1, 2)
        hidden = round(inp * expand_ratio)
        self.identity = stride == 1 and inp == oup
        self.stride = stride
        self.out_channels = oup
        layers = []
        if expand_ratio != 1:
            layers += [nn.Conv2d(inp, hidden, 1, 1, 0, bias=False), _norm_or_identity(norm, hidden),
                       nn.ReLU6(inplace=True)]
        layers += [nn.Conv2d(hidden, hidden, 3, stride, 1, groups=hidden, bias=False),
                   _norm_or_identity(norm, hidden), nn.ReLU6(inplace=True),
                   nn.Conv2d(hidden, oup, 1, 1, 0, bias=False), _norm_or_identity(norm, oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return run_seq(self.conv, x, residual=x if self.identity else None)[0]


class MobileNetV2Backbone(nn.Module):
    # t, c, n, s, output name
    CFGS = [[1, 16, 1, 1, ""], [6, 24, 2, 2, "m2"], [6, 32, 3, 2, "m3"], [6, 64, 4, 2, ""],
            [6, 96, 3, 1, "m4"], [6, 160, 3, 2, ""], [6, 320, 1, 1, "m5"]]

    def __init__(self, mcfg, in_channels=3, width_mult=1.0):
        super().__init__()
        self._out_features = list(mcfg.MOBILENETV2.OUT_FEATURES)
        norm = mcfg.MOBILENETV2.NORM
        freeze_at = mcfg.BACKBONE.FREEZE_AT
        div = 4 if width_mult == 0.1 else 8
        inp = _make_divisible(32 * width_mult, div)
        stem = nn.Sequential(nn.Conv2d(in_channels, inp, 3, 2, 1, bias=False),
                             _norm_or_identity(norm, inp), nn.ReLU6(inplace=True))
        if freeze_at >= 1:
            for p in stem.parameters():
                p.requires_grad = False
            stem = FrozenBatchNorm2d.convert_frozen_batchnorm(stem)
        layers = [stem]
        self.stage_name = [""]
        self._out_feature_channels, self._out_feature_strides = {}, {}
        stride, stage = 2, 2
        for t, c, n, s, name in self.CFGS:
            oup = _make_divisible(c * width_mult, div)
            stride *= s
            for i in range(n):
                layers.append(InvertedResidual(inp, oup, s if i == 0 else 1, t, norm))
                if stage <= freeze_at:
                    layers[-1].freeze()
                if name and i == n - 1:
                    self._out_feature_channels[name] = oup
                    self._out_feature_strides[name] = stride
                    stage += 1
                inp = oup
                self.stage_name.append(name if i == n - 1 else "")
        self.features = nn.Sequential(*layers)
        self._init_weights()

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
                if m.bias is not None:
                    m.bias.data.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def forward(self, x):
        out = {}
        for i, m in enumerate(self.features):
            x = run_seq(m, x)[0] if isinstance(m, nn.Sequential) else m(x)
            if self.stage_name[i] in self._out_features:
                out[self.stage_name[i]] = x
        return out

    def output_shape(self):
        return {n: ShapeSpec(self._out_feature_channels[n], self._out_feature_strides[n])
                for n in self._out_features}


def damp_residual_branches(module: nn.Module, scale: float = 0.25) -> int:
    """Scale the last norm of every residual branch by ``scale``.

    Random-init stand-in for pretrained weights: a FrozenBN (identity
    statistics) ResNet-101 grows its activations ~2x per block, which drives
    the ReviewKD/HCL loss to ~1e14 and the student off a cliff within a few
    steps.  Only applied when no checkpoint is loaded (synthetic runs, tests,
    benchmarks).  Returns the number of branches damped.
    """
    n = 0
    for m in module.modules():
        norm = None
        if isinstance(m, BottleneckBlock):
            norm = m.conv3.norm
        elif isinstance(m, BasicBlock):
            norm = m.conv2.norm
        elif isinstance(m, InvertedResidual) and m.identity:
            norm = m.conv[-1]
        if isinstance(norm, nn.BatchNorm2d) and norm.weight is not None:
            with torch.no_grad():
                norm.weight.mul_(scale)
            n += 1
    return n


# ----------------------------------------------------------------------------- FPN
class LastLevelMaxPool(nn.Module):
    num_levels = 1
    in_feature = "p5"

    def forward(self, x):
        return [F.max_pool2d(x, kernel_size=1, stride=2, padding=0)]


class FPN(nn.Module):
    def __init__(self, bottom_up, in_features, out_channels, norm="", top_block=None,
                 fuse_type="sum"):
        super().__init__()
        assert fuse_type in ("sum", "avg")
        shapes = bottom_up.output_shape()
        strides = [shapes[f].stride for f in in_features]
        in_channels = [shapes[f].channels for f in in_features]
        use_bias = norm == ""
        lateral, output = [], []
        for idx, ic in enumerate(in_channels):
            lconv = Conv2d(ic, out_channels, 1, bias=use_bias, norm=get_norm(norm, out_channels))
            oconv = Conv2d(out_channels, out_channels, 3, 1, 1, bias=use_bias,
                           norm=get_norm(norm, out_channels))
            c2_xavier_fill(lconv)
            c2_xavier_fill(oconv)
            stage = int(math.log2(strides[idx]))
            self.add_module(f"fpn_lateral{stage}", lconv)
            self.add_module(f"fpn_output{stage}", oconv)
            lateral.append(lconv)
            output.append(oconv)
        # plain lists (modules are registered above under Detectron2's names), deepest first
        self.lateral_convs = lateral[::-1]
        self.output_convs = output[::-1]
        self.top_block = top_block
        self.in_features = tuple(in_features)
        self.bottom_up = bottom_up
        self._out_feature_strides = {f"p{int(math.log2(s))}": s for s in strides}
        if top_block is not None:
            last = int(math.log2(strides[-1]))
            for s in range(last, last + top_block.num_levels):
                self._out_feature_strides[f"p{s + 1}"] = 2 ** (s + 1)
        self._out_features = list(self._out_feature_strides)
        self._out_feature_channels = {k: out_channels for k in self._out_features}
        self._size_divisibility = strides[-1]
        self._fuse_type = fuse_type

    @property
    def size_divisibility(self) -> int:
        return self._size_divisibility

    def forward(self, x):
        bu = self.bottom_up(x)
        results = []
        prev = self.lateral_convs[0](bu[self.in_features[-1]])
        results.append(self.output_convs[0](prev))
        for idx in range(1, len(self.lateral_convs)):
            feat = bu[self.in_features[-idx - 1]]
            top_down = F.interpolate(prev, scale_factor=2.0, mode="nearest")
            prev = self.lateral_convs[idx](feat, residual=top_down)  # lateral + top-down, one launch
            if self._fuse_type == "avg":
                prev = prev / 2
            results.insert(0, self.output_convs[idx](prev))
        if self.top_block is not None:
            results.extend(self.top_block(results[self._out_features.index(self.top_block.in_feature)]))
        return dict(zip(self._out_features, results))

    def output_shape(self):
        return {n: ShapeSpec(self._out_feature_channels[n], self._out_feature_strides[n])
                for n in self._out_features}


def _fpn(bottom_up, mcfg):
    return FPN(bottom_up, list(mcfg.FPN.IN_FEATURES), mcfg.FPN.OUT_CHANNELS, mcfg.FPN.NORM,
               LastLevelMaxPool(), mcfg.FPN.FUSE_TYPE)


BACKBONE_REGISTRY = {
    "build_resnet_backbone": build_resnet_backbone,
    "build_resnet_backbone_kd": build_resnet_backbone,
    "build_mobilenetv2_backbone": lambda m: MobileNetV2Backbone(m),
    "build_resnet_fpn_backbone": lambda m: _fpn(build_resnet_backbone(m), m),
    "build_resnet_fpn_backbone_kd": lambda m: _fpn(build_resnet_backbone(m), m),
    "build_mobilenetv2_fpn_backbone": lambda m: _fpn(MobileNetV2Backbone(m), m),
}


def build_backbone(mcfg):
    name = mcfg.BACKBONE.NAME
    if name not in BACKBONE_REGISTRY:
        raise NotImplementedError(f"backbone {name!r}")
    bb = BACKBONE_REGISTRY[name](mcfg)
    if not hasattr(bb, "size_divisibility"):
        bb.size_divisibility = 0
    return bb
