"""CIFAR MobileNetV2 (``mobile_half``: T=6, width 0.5).

Layout follows `mdistiller/models/cifar/mobilenetv2.py:26-217` (the stray
``print(T, width_mult)`` of `:117`, SURVEY D19, is dropped).  Pointwise convs
run on the MFMA implicit-GEMM kernel (1x1 = plain GEMM over pixels); the
depthwise 3x3 goes to the dedicated depthwise kernel.

Channel padding (round 3): the native kernels move 8 channels (16 bytes) per
vector, and width 0.5 makes one stage 12 channels wide.  Those layers are
built PHYSICALLY padded to the next multiple of 8 (12 -> 16): zero weight
rows / columns, BN gamma = beta = 0 on the pad channels.  Pad channels then
carry exact zeros forward (conv rows of zeros, scale 0 / shift 0), receive
exactly zero gradients backward (their BN scale is 0, the consumer's weight
columns are 0, relu'(0) = 0), so SGD with weight decay keeps them at zero
forever: the network is the reference's, run on 16-byte-aligned tensors with
no MIOpen fallback.  ``state_dict`` / ``load_state_dict`` see the reference
(unpadded) shapes, and the feature maps handed to distillers are sliced to
the real channels.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops.nn import grad_fork, pool_linear
from .._base import ModelBase
from .._seq import run_seq


def conv_bn(inp, oup, stride):
    return nn.Sequential(nn.Conv2d(inp, oup, 3, stride, 1, bias=False), nn.BatchNorm2d(oup))


def conv_1x1_bn(inp, oup):
    return nn.Sequential(nn.Conv2d(inp, oup, 1, 1, 0, bias=False), nn.BatchNorm2d(oup),
                         nn.ReLU(inplace=True))


def _phys(c: int) -> int:
    return (c + 7) // 8 * 8


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        assert stride in (1, 2)
        self.blockname = None
        self.stride = stride
        self.use_res_connect = stride == 1 and inp == oup
        hid = inp * expand_ratio
        # real widths (reference layout) and physical ones (multiples of 8)
        self.real = (inp, hid, oup)
        self.conv = nn.Sequential(
            nn.Conv2d(_phys(inp), hid, 1, 1, 0, bias=False), nn.BatchNorm2d(hid), nn.ReLU(inplace=True),
            nn.Conv2d(hid, hid, 3, stride, 1, groups=hid, bias=False), nn.BatchNorm2d(hid),
            nn.ReLU(inplace=True),
            nn.Conv2d(hid, _phys(oup), 1, 1, 0, bias=False), nn.BatchNorm2d(_phys(oup)),
        )
        self.names = ["0", "1", "2", "3", "4", "5", "6", "7"]

    @torch.no_grad()
    def zero_padding(self):
        inp, _, oup = self.real
        self.conv[0].weight[:, inp:].zero_()
        self.conv[6].weight[oup:].zero_()
        bn = self.conv[7]
        bn.weight[oup:].zero_()
        bn.bias[oup:].zero_()
        bn.running_mean[oup:].zero_()
        bn.running_var[oup:].fill_(1.0)

    # the reference's (unpadded) parameter shapes on the state_dict boundary
    def _pad_map(self):
        inp, _, oup = self.real
        return {"conv.0.weight": (None, inp), "conv.6.weight": (oup, None),
                "conv.7.weight": (oup,), "conv.7.bias": (oup,), "conv.7.running_mean": (oup,),
                "conv.7.running_var": (oup,)}

    def forward(self, x, final_act=None):
        """``final_act``: also apply this activation to the block output and
        return ``(activated, linear)`` from the same fused launch."""
        res = x if self.use_res_connect else None
        # x feeds the expansion conv and the residual add: their input
        # gradients are summed in the native backward (GradFork)
        fork = grad_fork(x) if res is not None else None
        if final_act is None:
            return run_seq(self.conv, x, residual=res, fork=fork)[0]
        return run_seq(self.conv, x, residual=res, want_preact=True, final_act=final_act,
                       fork=fork)


class _Group(nn.Module):
    """``blocks[i](relu?(x)) -> blocks[j](...)`` as one staged layer."""

    def __init__(self, *blocks, phys_in=None, real_out=None):
        super().__init__()
        self.blocks = blocks
        self.phys_in, self.real_out = phys_in, real_out

    def forward(self, x):
        # staged API: tensors between stages carry the REAL channels; a stage
        # whose first layer is physically padded gets zero channels appended
        if self.phys_in is not None and x.shape[1] < self.phys_in:
            x = F.pad(x, (0, 0, 0, 0, 0, self.phys_in - x.shape[1]))
        for b in self.blocks:
            x = b(x)
        if self.real_out is not None and x.shape[1] > self.real_out:
            x = x[:, :self.real_out]
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
        self.conv2 = conv_1x1_bn(_phys(input_channel), self.last_channel)
        self._conv2_in = input_channel
        self.classifier = nn.Sequential(nn.Linear(self.last_channel, feature_dim))
        self._pool_k = input_size // (32 // 2)
        self.avgpool = nn.AvgPool2d(self._pool_k, ceil_mode=True)
        self._initialize_weights()
        self._zero_padding()
        self.stage_channels = [int(c * width_mult) for c in (32, 24, 32, 96, 320)]
        # real channels of the five feature maps (f0 .. f4)
        self._feat_c = [int(32 * width_mult)] + [int(self.interverted_residual_setting[i][1] * width_mult)
                                                 for i in (1, 2, 4, 6)]
        self._register_state_dict_hook(MobileNetV2._sd_slice)
        self._register_load_state_dict_pre_hook(self._sd_pad)

    @torch.no_grad()
    def _zero_padding(self):
        for blk in self._irs():
            blk.zero_padding()
        self.conv2[0].weight[:, self._conv2_in:].zero_()

    def _irs(self):
        return [m for m in self.modules() if isinstance(m, InvertedResidual)]

    def _pad_entries(self):
        out = {}
        for name, m in self.named_modules():
            if isinstance(m, InvertedResidual):
                for k, v in m._pad_map().items():
                    out[f"{name}.{k}"] = v
        out["conv2.0.weight"] = (None, self._conv2_in)
        return out

    @staticmethod
    def _sd_slice(module, sd, prefix, local_metadata):
        for k, spec in module._pad_entries().items():
            key = prefix + k
            if key not in sd:
                continue
            t = sd[key]
            if len(spec) == 1:
                t = t[:spec[0]]
            elif spec[0] is not None:
                t = t[:spec[0]]
            else:
                t = t[:, :spec[1]]
            sd[key] = t.clone()
        return sd

    def _sd_pad(self, sd, prefix, *args):
        own = dict(self.named_parameters())
        own.update(dict(self.named_buffers()))
        for k in self._pad_entries():
            key = prefix + k
            if key not in sd or k not in own:
                continue
            t, ref = sd[key], own[k]
            if t.shape == ref.shape:
                continue
            z = torch.zeros_like(ref, device=t.device, dtype=t.dtype)
            if k.endswith("running_var"):
                z.fill_(1.0)
            z[tuple(slice(0, n) for n in t.shape)] = t
            sd[key] = z

    def get_bn_before_relu(self):
        return [self.blocks[1][-1].conv[-1], self.blocks[2][-1].conv[-1],
                self.blocks[4][-1].conv[-1], self.blocks[6][-1].conv[-1]]

    def forward_stem(self, x):
        return run_seq(self.conv1, x)[0]

    def get_layers(self):
        b = self.blocks
        fc = self._feat_c

        def cin(blk):
            return blk[0].conv[0].in_channels
        return nn.Sequential(_Group(b[0], b[1], phys_in=cin(b[0]), real_out=fc[1]),
                             _Group(b[2], phys_in=cin(b[2]), real_out=fc[2]),
                             _Group(b[3], b[4], phys_in=cin(b[3]), real_out=fc[3]),
                             _Group(b[5], b[6], phys_in=cin(b[5]), real_out=fc[4]))

    def forward_pool(self, x):
        if x.shape[1] < self.conv2[0].in_channels:
            x = F.pad(x, (0, 0, 0, 0, 0, self.conv2[0].in_channels - x.shape[1]))
        out = run_seq(self.conv2, F.relu(x))[0]
        if not self.remove_avg:
            out = self.avgpool(out)
        return out.reshape(out.size(0), -1)

    def get_head(self):
        return self.classifier

    @staticmethod
    def _stage(seq, x):
        """A run of inverted residuals whose output feeds a ReLU: the last
        block returns (relu(out), out) from one fused launch."""
        for blk in list(seq)[:-1]:
            x = blk(x)
        return seq[-1](x, final_act="relu")

    def forward(self, x):
        # the reference applies F.relu to f0..f4 before their consumers; here
        # each stage's last conv emits both tensors in one launch
        a0, f0 = run_seq(self.conv1, x, want_preact=True, final_act="relu")
        out = self.blocks[0](a0)
        a1, f1 = self._stage(self.blocks[1], out)
        a2, f2 = self._stage(self.blocks[2], a1)
        out = self.blocks[3](a2)
        a3, f3 = self._stage(self.blocks[4], out)
        out = self.blocks[5](a3)
        a4, f4 = self._stage(self.blocks[6], out)
        out = run_seq(self.conv2, a4)[0]
        if not self.remove_avg and out.shape[-1] == out.shape[-2] == self._pool_k:
            # a global pool: the fused pool + classifier (same values as
            # AvgPool2d + Linear, native backward)
            avg, logits = pool_linear(out, self.classifier[0], self._pool_k)
        else:
            if not self.remove_avg:
                out = self.avgpool(out)
            avg = out.reshape(out.size(0), -1)
            logits = self.classifier(avg)

        def real(ts):
            return [t if t.shape[1] == c else t[:, :c] for t, c in zip(ts, self._feat_c)]
        return logits, {
            "feats": real((a0, a1, a2, a3, a4)),
            "preact_feats": real((f0, f1, f2, f3, f4)),
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
