"""CIFAR ShuffleNet V1 (g=3) and V2 (1x).

Layouts follow `mdistiller/models/cifar/ShuffleNetv1.py:7-169` and
`ShuffleNetv2.py:7-233`.  ShuffleV2's head uses a global average pool instead
of ``avg_pool2d(out, 4)``: identical on 32x32 inputs (4x4 map) and correct on
64x64 Tiny-ImageNet inputs, where the reference produces 4096 features for a
1024-wide classifier.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import (conv_bn_act, channel_gather, channel_shuffle, grad_fork, pool_linear,
                       shuffle_tail, ChannelRoute, gather2)
from .._base import ModelBase, PreactStage
from .resnet import Stage


class ShuffleBlock(nn.Module):
    def __init__(self, groups=2):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        return channel_shuffle(x, self.groups)


# ----------------------------------------------------------------------------- V1
def _ceil8(c: int) -> int:
    return (c + 7) // 8 * 8


class BottleneckV1(nn.Module):
    """ShuffleNetV1 unit with PHYSICALLY padded groups (round 3).

    The bottleneck width ``mid`` splits into groups of mid/g1 (conv1, g1 = 1 for
    the first unit) and mid/g (conv3) channels -- 18 or 20 on CIFAR, which the
    16-byte-vector kernels cannot address.  Each group is padded to a multiple
    of 8 with zero weight rows / columns and BN gamma = beta = 0: pad channels
    carry exact zeros forward, get exactly zero gradients (BN scale 0, zero
    consumer columns, gather maps that never read them), and so stay zero under
    SGD + weight decay.  The channel shuffle between the two layouts is one
    gather (``channel_gather``: conv1's padded groups -> shuffled order ->
    conv3's padded groups), and conv1 / conv3 run as compact grouped GEMMs.
    ``state_dict`` shows the reference's (unpadded) shapes
    (`mdistiller/models/cifar/ShuffleNetv1.py:19-63`).
    """

    def __init__(self, in_planes, out_planes, stride, groups, is_last=False):
        super().__init__()
        self.is_last = is_last
        self._need_preact = True
        self.stride = stride
        mid = int(out_planes / 4)
        g = 1 if in_planes == 24 else groups
        m1, m3 = mid // g, mid // groups
        m1p, m3p = _ceil8(m1), _ceil8(m3)
        self.real = dict(mid=mid, g1=g, g3=groups, m1=m1, m3=m3, m1p=m1p, m3p=m3p, out=out_planes)
        self.conv1 = nn.Conv2d(in_planes, g * m1p, 1, groups=g, bias=False)
        self.bn1 = nn.BatchNorm2d(g * m1p)
        self.shuffle1 = ShuffleBlock(groups=g)
        self.conv2 = nn.Conv2d(groups * m3p, groups * m3p, 3, stride, 1, groups=groups * m3p, bias=False)
        self.bn2 = nn.BatchNorm2d(groups * m3p)
        self.conv3 = nn.Conv2d(groups * m3p, out_planes, 1, groups=groups, bias=False)
        self.bn3 = nn.BatchNorm2d(out_planes)
        self.shortcut = nn.Sequential()
        if stride == 2:
            self.shortcut = nn.Sequential(nn.AvgPool2d(3, stride=2, padding=1))
        # conv3-layout channel k*m3p + t  <-  shuffled real channel j = k*m3 + t
        #                                 <-  conv1-layout channel (j % g)*m1p + j // g
        fmap = [-1] * (groups * m3p)
        for k in range(groups):
            for t in range(m3):
                j = k * m3 + t
                fmap[k * m3p + t] = (j % g) * m1p + j // g
        bmap = [-1] * (g * m1p)
        for c, src in enumerate(fmap):
            if src >= 0:
                bmap[src] = c
        self.register_buffer("_fmap", torch.tensor(fmap, dtype=torch.int32), persistent=False)
        self.register_buffer("_bmap", torch.tensor(bmap, dtype=torch.int32), persistent=False)
        # physical index of every real channel (reference order)
        self._idx1 = [(r // m1) * m1p + r % m1 for r in range(mid)]
        self._idx3 = [(j // m3) * m3p + j % m3 for j in range(mid)]
        self._init_real()

    @torch.no_grad()
    def _init_real(self):
        R = self.real
        # the reference's default init on the reference shapes, then placed
        ref3 = nn.Conv2d(R["mid"], R["out"], 1, groups=R["g3"], bias=False)
        self.conv3.weight.zero_()
        self.conv3.weight[:, :R["m3"]].copy_(ref3.weight)
        keep1 = torch.zeros(self.conv1.out_channels, dtype=torch.bool)
        keep1[self._idx1] = True
        keep3 = torch.zeros(self.conv2.out_channels, dtype=torch.bool)
        keep3[self._idx3] = True
        self.conv1.weight[~keep1] = 0
        self.conv2.weight[~keep3] = 0
        for bn, keep in ((self.bn1, keep1), (self.bn2, keep3)):
            bn.weight[~keep] = 0
            bn.bias[~keep] = 0

    def _pad_specs(self):
        """state_dict key -> (dim, physical indices of the real entries)."""
        i1, i3 = self._idx1, self._idx3
        out = {"conv1.weight": (0, i1), "conv2.weight": (0, i3),
               "conv3.weight": (1, list(range(self.real["m3"])))}
        for k in ("weight", "bias", "running_mean", "running_var"):
            out[f"bn1.{k}"] = (0, i1)
            out[f"bn2.{k}"] = (0, i3)
        return out

    def forward(self, x):
        # x feeds conv1 and the residual (stride 1) or the pooled shortcut
        # (stride 2); their gradients are summed in conv1's dgrad epilogue
        # (GradFork) instead of an autograd add
        fork = grad_fork(x)
        out, _ = conv_bn_act(x, self.conv1, self.bn1, "relu", fork=fork)
        out = channel_gather(out, self._fmap, self._bmap)
        out, _ = conv_bn_act(out, self.conv2, self.bn2, "relu")
        if self.stride == 2:
            out, _ = conv_bn_act(out, self.conv3, self.bn3, "none")
            # cat([out, avgpool3x3s2(x)]) + relu: one native pass (ops.nn.shuffle_tail)
            return shuffle_tail(out, x, fork)
        return conv_bn_act(out, self.conv3, self.bn3, "relu", residual=x,
                           want_preact=self.is_last and self._need_preact, res_fork=fork)


class ShuffleNet(nn.Module, ModelBase):
    def __init__(self, cfg, num_classes=10):
        super().__init__()
        out_planes, num_blocks, groups = cfg["out_planes"], cfg["num_blocks"], cfg["groups"]
        self.conv1 = nn.Conv2d(3, 24, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(24)
        self.in_planes = 24
        self.layer1 = self._make_layer(out_planes[0], num_blocks[0], groups)
        self.layer2 = self._make_layer(out_planes[1], num_blocks[1], groups)
        self.layer3 = self._make_layer(out_planes[2], num_blocks[2], groups)
        self.linear = nn.Linear(out_planes[2], num_classes)
        self.stage_channels = [24] + list(out_planes)
        self._register_state_dict_hook(ShuffleNet._sd_slice)
        self._register_load_state_dict_pre_hook(self._sd_pad)

    def _pad_entries(self):
        out = {}
        for name, m in self.named_modules():
            if isinstance(m, BottleneckV1):
                for k, v in m._pad_specs().items():
                    out[f"{name}.{k}"] = v
        return out

    @staticmethod
    def _sd_slice(module, sd, prefix, local_metadata):
        # physical (group-padded) tensors -> the reference's shapes
        for k, (dim, idx) in module._pad_entries().items():
            key = prefix + k
            if key in sd:
                t = sd[key]
                sd[key] = t.index_select(dim, torch.tensor(idx, device=t.device)).clone()
        return sd

    def _sd_pad(self, sd, prefix, *args):
        own = dict(self.named_parameters())
        own.update(dict(self.named_buffers()))
        for k, (dim, idx) in self._pad_entries().items():
            key = prefix + k
            if key not in sd or k not in own or sd[key].shape == own[k].shape:
                continue
            t, ref = sd[key], own[k]
            z = torch.zeros(ref.shape, device=t.device, dtype=t.dtype)
            if k.endswith("running_var"):
                z.fill_(1.0)
            z.index_copy_(dim, torch.tensor(idx, device=t.device), t)
            sd[key] = z

    def _make_layer(self, out_planes, num_blocks, groups):
        layers = []
        for i in range(num_blocks):
            stride = 2 if i == 0 else 1
            cat_planes = self.in_planes if i == 0 else 0
            layers.append(BottleneckV1(self.in_planes, out_planes - cat_planes, stride, groups,
                                       is_last=(i == num_blocks - 1)))
            self.in_planes = out_planes
        return Stage(*layers)

    def get_bn_before_relu(self):
        raise NotImplementedError('ShuffleNet is not supported as an "Overhaul" (OFD) teacher')

    def forward_stem(self, x):
        return self.bn1(self.conv1(x))

    def get_layers(self):
        return nn.Sequential(PreactStage(self.layer1), PreactStage(self.layer2), PreactStage(self.layer3))

    def forward_pool(self, x):
        out = F.adaptive_avg_pool2d(F.relu(x), 1)
        return out.reshape(out.size(0), -1)

    def get_head(self):
        return self.linear

    def forward(self, x):
        out, f0_pre = conv_bn_act(x, self.conv1, self.bn1, "relu", want_preact=True)
        f0 = out
        out, f1_pre = self.layer1(out)
        f1 = out
        out, f2_pre = self.layer2(out)
        f2 = out
        out, f3_pre = self.layer3(out)
        f3 = out
        avg, logits = pool_linear(out, self.linear)
        return logits, {"feats": [f0, f1, f2, f3],
                                  "preact_feats": [f0_pre, f1_pre, f2_pre, f3_pre],
                                  "pooled_feat": avg}


def ShuffleV1(**kw):
    return ShuffleNet({"out_planes": [240, 480, 960], "num_blocks": [4, 8, 4], "groups": 3}, **kw)


# ----------------------------------------------------------------------------- V2
# ShuffleNetV2 (reference ShuffleNetv2.py:29-113) with channel-PADDED halves.
# The 1x width has 58 / 116 channels per half at stages 1-2, which the
# 16-byte-vector kernels cannot address; each half is padded to a multiple of
# 8 (64 / 120) with zero weights and BN gamma = beta = 0, so pad channels carry
# exact zeros and get exactly zero gradients (the ShuffleV1 argument above).
# Between units the activation is a PAIR of tensors: the two halves the next
# unit's split produces, each [N, cp] -- so the split is free, and the concat +
# channel shuffle + split is ONE routing launch per output half
# (``ops.nn.gather2``), instead of cat + shuffle copies.  ``state_dict`` has the
# reference's shapes.
class SplitBlock(nn.Module):
    def __init__(self, ratio):
        super().__init__()
        self.ratio = ratio

    def forward(self, x):
        c = int(x.size(1) * self.ratio)
        return x[:, :c, :, :], x[:, c:, :, :]


class _Pair(tuple):
    """(A, B): the logical first / second halves of a unit's output, each
    channel-padded to cp (the real channels first)."""


def _shuffle_routes(c, cp, src_a, src_b):
    """Routes of ``split(shuffle(cat([a, b])))``: logical channel 2i = a_i,
    2i+1 = b_i (a, b: c real channels each), cut into two halves of c, each
    padded to cp.  Sources: a = ``src_a`` (index, channel offset), b likewise."""
    logical = []
    for i in range(c):
        logical.append((src_a[0], src_a[1] + i))
        logical.append((src_b[0], src_b[1] + i))
    half = lambda lo: logical[lo:lo + c] + [None] * (cp - c)  # noqa: E731
    return [half(0), half(c)]


def _pair_to_logical_routes(c, cp):
    """(A, B) -> the logical tensor [N, 2c]."""
    return [[(0, i) for i in range(c)] + [(1, i) for i in range(c)]]


class BasicBlockV2(nn.Module):
    def __init__(self, in_channels, split_ratio=0.5, is_last=False):
        super().__init__()
        self.is_last = is_last
        self._need_preact = True
        c = int(in_channels * split_ratio)
        cp = _ceil8(c)
        self.c, self.cp = c, cp
        self.conv1 = nn.Conv2d(cp, cp, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cp)
        self.conv2 = nn.Conv2d(cp, cp, 3, 1, 1, groups=cp, bias=False)
        self.bn2 = nn.BatchNorm2d(cp)
        self.conv3 = nn.Conv2d(cp, cp, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cp)
        # out = (A', B') from sources (A = the unit's first half, y = branch output)
        self.route = ChannelRoute(_shuffle_routes(c, cp, (0, 0), (1, 0)), [cp, cp])
        self.route_log = ChannelRoute(_pair_to_logical_routes(c, cp), [cp, cp])
        self.route_pre = ChannelRoute([[r for pair in zip([(0, i) for i in range(c)],
                                                           [(1, i) for i in range(c)]) for r in pair]],
                                      [cp, cp])
        self._init_real()

    @torch.no_grad()
    def _init_real(self):
        c = self.c
        ref = [nn.Conv2d(c, c, 1, bias=False), nn.Conv2d(c, c, 3, 1, 1, groups=c, bias=False),
               nn.Conv2d(c, c, 1, bias=False)]
        for conv, r in zip((self.conv1, self.conv2, self.conv3), ref):
            conv.weight.zero_()
            conv.weight[:c, :r.weight.shape[1]].copy_(r.weight)
        for bn in (self.bn1, self.bn2, self.bn3):
            bn.weight[c:] = 0
            bn.bias[c:] = 0

    def _pad_specs(self):
        r = list(range(self.c))
        out = {"conv1.weight": [(0, r), (1, r)], "conv2.weight": [(0, r)],
               "conv3.weight": [(0, r), (1, r)]}
        for bn in ("bn1", "bn2", "bn3"):
            for k in ("weight", "bias", "running_mean", "running_var"):
                out[f"{bn}.{k}"] = [(0, r)]
        return out

    def forward(self, x):
        a, b = x
        out, _ = conv_bn_act(b, self.conv1, self.bn1, "relu")
        out, _ = conv_bn_act(out, self.conv2, self.bn2, "none")
        want = self.is_last and self._need_preact
        out, pre = conv_bn_act(out, self.conv3, self.bn3, "relu", want_preact=want)
        nxt = _Pair(gather2(self.route, a, out))
        # preact in the same (shuffled) channel order as the logical output
        preact = gather2(self.route_pre, a, pre) if want else None
        return nxt, preact


class DownBlock(nn.Module):
    def __init__(self, in_channels, out_channels, in_pad=None):
        """``in_pad`` = (c, cp): the input is a padded pair of two c-channel
        halves (logical channel i -> physical i, c + i -> cp + i after
        concatenation); None: a plain tensor of ``in_channels``."""
        super().__init__()
        self._need_preact = True
        mid = out_channels // 2
        mp = _ceil8(mid)
        if in_pad is None:
            in_p, in_idx = in_channels, list(range(in_channels))
        else:
            c, cp = in_pad
            in_p, in_idx = 2 * cp, list(range(c)) + [cp + i for i in range(c)]
            self.route_in = ChannelRoute([[(0, i) for i in range(cp)] + [(1, i) for i in range(cp)]],
                                         [cp, cp])
        self.in_pad = in_pad
        self.mid, self.mp, self.in_idx = mid, mp, in_idx
        self.conv1 = nn.Conv2d(in_p, in_p, 3, 2, 1, groups=in_p, bias=False)
        self.bn1 = nn.BatchNorm2d(in_p)
        self.conv2 = nn.Conv2d(in_p, mp, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(mp)
        self.conv3 = nn.Conv2d(in_p, mp, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(mp)
        self.conv4 = nn.Conv2d(mp, mp, 3, 2, 1, groups=mp, bias=False)
        self.bn4 = nn.BatchNorm2d(mp)
        self.conv5 = nn.Conv2d(mp, mp, 1, bias=False)
        self.bn5 = nn.BatchNorm2d(mp)
        self.route = ChannelRoute(_shuffle_routes(mid, mp, (0, 0), (1, 0)), [mp, mp])
        self._init_real(in_channels)

    @torch.no_grad()
    def _init_real(self, cin):
        mid, idx = self.mid, torch.tensor(self.in_idx)
        r1 = nn.Conv2d(cin, cin, 3, 2, 1, groups=cin, bias=False)
        r2, r3 = nn.Conv2d(cin, mid, 1, bias=False), nn.Conv2d(cin, mid, 1, bias=False)
        r4, r5 = nn.Conv2d(mid, mid, 3, 2, 1, groups=mid, bias=False), nn.Conv2d(mid, mid, 1, bias=False)
        for conv in (self.conv1, self.conv2, self.conv3, self.conv4, self.conv5):
            conv.weight.zero_()
        self.conv1.weight[idx] = r1.weight
        self.conv2.weight[:mid, idx] = r2.weight[:, :, 0, 0].unsqueeze(-1).unsqueeze(-1)
        self.conv3.weight[:mid, idx] = r3.weight[:, :, 0, 0].unsqueeze(-1).unsqueeze(-1)
        self.conv4.weight[:mid] = r4.weight
        self.conv5.weight[:mid, :mid] = r5.weight
        keep_in = torch.zeros(self.conv1.out_channels, dtype=torch.bool)
        keep_in[idx] = True
        self.bn1.weight[~keep_in] = 0
        self.bn1.bias[~keep_in] = 0
        for bn in (self.bn2, self.bn3, self.bn4, self.bn5):
            bn.weight[mid:] = 0
            bn.bias[mid:] = 0

    def _pad_specs(self):
        i, r = self.in_idx, list(range(self.mid))
        out = {"conv1.weight": [(0, i)], "conv2.weight": [(0, r), (1, i)],
               "conv3.weight": [(0, r), (1, i)], "conv4.weight": [(0, r)],
               "conv5.weight": [(0, r), (1, r)]}
        for bn, ix in (("bn1", i), ("bn2", r), ("bn3", r), ("bn4", r), ("bn5", r)):
            for k in ("weight", "bias", "running_mean", "running_var"):
                out[f"{bn}.{k}"] = [(0, ix)]
        return out

    def forward(self, x):
        if isinstance(x, tuple):
            x = gather2(self.route_in, x[0], x[1])
        o1, _ = conv_bn_act(x, self.conv1, self.bn1, "none")
        o1, _ = conv_bn_act(o1, self.conv2, self.bn2, "relu")
        o2, _ = conv_bn_act(x, self.conv3, self.bn3, "relu")
        o2, _ = conv_bn_act(o2, self.conv4, self.bn4, "none")
        o2, _ = conv_bn_act(o2, self.conv5, self.bn5, "relu")
        out = _Pair(gather2(self.route, o1, o2))
        return out, None


class ShuffleV2Stage(nn.Sequential):
    """A stage on padded pairs.  ``forward(pair or tensor)``; the staged API
    (a logical tensor in) gets the logical (out, preact) back."""

    def __init__(self, *blocks, c, cp, in_pad=None):
        super().__init__(*blocks)
        self.c, self.cp, self.in_pad = c, cp, in_pad
        self.route_log = ChannelRoute(_pair_to_logical_routes(c, cp), [cp, cp])
        if in_pad is not None:
            ci, cip = in_pad
            self.route_split = ChannelRoute([[(0, i) for i in range(ci)] + [None] * (cip - ci),
                                             [(0, ci + i) for i in range(ci)] + [None] * (cip - ci)],
                                            [2 * ci])

    def logical(self, pair):
        return gather2(self.route_log, pair[0], pair[1])

    def run(self, x):
        """Model forward: x = the stem tensor (stage 1) or the previous stage's
        pair -> (pair, logical preact or None)."""
        pre = None
        for blk in self:
            x, pre = blk(x)
        return x, pre

    def forward(self, x):
        """Staged API: the LOGICAL activated input -> logical (out, preact)."""
        if self.in_pad is not None:
            x = _Pair(gather2(self.route_split, x))
        x, pre = self.run(x)
        return self.logical(x), pre


def _ceil8_v2(c):
    return (c + 7) // 8 * 8


configs_v2 = {
    0.2: {"out_channels": (40, 80, 160, 512), "num_blocks": (3, 3, 3)},
    0.3: {"out_channels": (40, 80, 160, 512), "num_blocks": (3, 7, 3)},
    0.5: {"out_channels": (48, 96, 192, 1024), "num_blocks": (3, 7, 3)},
    1: {"out_channels": (116, 232, 464, 1024), "num_blocks": (3, 7, 3)},
    1.5: {"out_channels": (176, 352, 704, 1024), "num_blocks": (3, 7, 3)},
    2: {"out_channels": (224, 488, 976, 2048), "num_blocks": (3, 7, 3)},
}


class ShuffleNetV2(nn.Module, ModelBase):
    def __init__(self, net_size, num_classes=10):
        super().__init__()
        out_channels = configs_v2[net_size]["out_channels"]
        num_blocks = configs_v2[net_size]["num_blocks"]
        self.conv1 = nn.Conv2d(3, 24, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(24)
        self.in_channels = 24
        self._in_pad = None
        self.layer1 = self._make_layer(out_channels[0], num_blocks[0])
        self.layer2 = self._make_layer(out_channels[1], num_blocks[1])
        self.layer3 = self._make_layer(out_channels[2], num_blocks[2])
        self.conv2 = nn.Conv2d(out_channels[2], out_channels[3], 1, 1, 0, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels[3])
        self.linear = nn.Linear(out_channels[3], num_classes)
        self.stage_channels = out_channels
        self._register_state_dict_hook(ShuffleNetV2._sd_slice)
        self._register_load_state_dict_pre_hook(self._sd_pad)

    def _make_layer(self, out_channels, num_blocks):
        c = out_channels // 2
        cp = _ceil8_v2(c)
        layers = [DownBlock(self.in_channels, out_channels, in_pad=self._in_pad)]
        for i in range(num_blocks):
            layers.append(BasicBlockV2(out_channels, is_last=(i == num_blocks - 1)))
        stage = ShuffleV2Stage(*layers, c=c, cp=cp, in_pad=self._in_pad)
        self.in_channels = out_channels
        self._in_pad = (c, cp)
        return stage

    # reference-shaped state_dict ------------------------------------------------
    def _pad_entries(self):
        out = {}
        for name, m in self.named_modules():
            if isinstance(m, (BasicBlockV2, DownBlock)):
                for k, v in m._pad_specs().items():
                    out[f"{name}.{k}"] = v
        return out

    @staticmethod
    def _sd_slice(module, sd, prefix, local_metadata):
        for k, specs in module._pad_entries().items():
            key = prefix + k
            if key in sd:
                t = sd[key]
                for dim, idx in specs:
                    t = t.index_select(dim, torch.tensor(idx, device=t.device))
                sd[key] = t.clone()
        return sd

    def _sd_pad(self, sd, prefix, *args):
        own = dict(self.named_parameters())
        own.update(dict(self.named_buffers()))
        for k, specs in self._pad_entries().items():
            key = prefix + k
            if key not in sd or k not in own or sd[key].shape == own[k].shape:
                continue
            t, ref = sd[key], own[k]
            z = torch.zeros(ref.shape, device=t.device, dtype=t.dtype)
            if k.endswith("running_var"):
                z.fill_(1.0)
            if len(specs) == 1:
                dim, idx = specs[0]
                z.index_copy_(dim, torch.tensor(idx, device=t.device), t)
            else:
                (d0, i0), (d1, i1) = specs
                rows = torch.zeros((ref.shape[0],) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
                rows.index_copy_(d0, torch.tensor(i0, device=t.device), t)
                z.index_copy_(d1, torch.tensor(i1, device=t.device), rows)
            sd[key] = z

    def get_bn_before_relu(self):
        raise NotImplementedError('ShuffleNetV2 is not supported as an "Overhaul" (OFD) teacher')

    def get_stage_channels(self):
        return [24] + list(self.stage_channels[:-1])

    def forward_stem(self, x):
        return self.bn1(self.conv1(x))

    def get_layers(self):
        return nn.Sequential(PreactStage(self.layer1), PreactStage(self.layer2), PreactStage(self.layer3))

    def _head(self, out):
        out, _ = conv_bn_act(out, self.conv2, self.bn2, "relu")
        return F.adaptive_avg_pool2d(out, 1).reshape(out.size(0), -1)

    def forward_pool(self, x):
        return self._head(F.relu(x))

    def get_head(self):
        return self.linear

    def forward(self, x):
        out, f0_pre = conv_bn_act(x, self.conv1, self.bn1, "relu", want_preact=True)
        feats, pres = [out], [f0_pre]
        for layer in (self.layer1, self.layer2, self.layer3):
            out, pre = layer.run(out)
            feats.append(layer.logical(out))
            pres.append(pre if pre is not None else feats[-1])
        out, _ = conv_bn_act(feats[-1], self.conv2, self.bn2, "relu")
        avg, logits = pool_linear(out, self.linear)  # global pool + FC, one native pass
        return logits, {"feats": feats, "preact_feats": pres, "pooled_feat": avg}


def ShuffleV2(**kw):
    return ShuffleNetV2(net_size=1, **kw)
