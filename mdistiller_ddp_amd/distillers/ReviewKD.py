"""Distilling Knowledge via Knowledge Review, CVPR 2021
(reference `distillers/ReviewKD.py:31-144`).

The student's stage features plus the pooled vector are fused deepest-first
by a chain of attention-based fusion (ABF) modules; each output is matched to
the teacher's pre-ReLU stage feature (plus pooled) with the hierarchical
context loss (HCL: MSE at full resolution + 4/2/1 average-pooled pyramid).

Feature lists use the stem-inclusive model contract: student
``feats[1:]`` (or ``preact_feats[1:]`` with ``STU_PREACT``) + pooled, teacher
``preact_feats[1:]`` + pooled, so the shipped ``REVIEWKD.{SHAPES,
IN_CHANNELS}`` lists line up (the reference's fork misaligns them, D6).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL
from ..ops.nn import conv_bn_act


class _ABFFuse(torch.autograd.Function):
    """``x * s0 + up(y) * s1``, ``(s0, s1) = sigmoid(att_conv([x; up(y)]))`` on the
    fused HIP kernels (``ops/csrc/reviewkd.hip``): no upsampled copy of ``y``,
    no concat, no separate 1x1 conv / sigmoid / blend launches."""

    @staticmethod
    def forward(ctx, x, y, weight, bias):
        from ..ops import _ext
        N, C, h, w = x.shape
        hy, wy = y.shape[2], y.shape[3]
        x = x.contiguous(memory_format=torch.channels_last)
        y = y.to(x.dtype).contiguous(memory_format=torch.channels_last)
        out = torch.empty_like(x, memory_format=torch.channels_last)
        att = torch.empty(N * h * w * 2, dtype=torch.float32, device=x.device)
        wt = weight.detach().reshape(2, 2 * C).contiguous()
        _ext.call("mda_abf_fwd", x, y, wt, bias.detach() if bias is not None else None, out, att,
                  N, h, w, hy, wy, C)
        ctx.save_for_backward(x, y, att, weight, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        import ctypes
        from ..ops import _ext
        x, y, att, weight, bias = ctx.saved_tensors
        N, C, h, w = x.shape
        hy, wy = y.shape[2], y.shape[3]
        dout = dout.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dy = torch.empty_like(y, memory_format=torch.channels_last) if ctx.needs_input_grad[1] else None
        dyup = torch.empty(N * h * w * C, dtype=torch.float32, device=x.device)
        nb = ctypes.c_int64(0)
        _ext.call("mda_abf_bwd_blocks", N, h, w, C, nb)
        part = torch.empty(nb.value * (4 * C + 2), dtype=torch.float32, device=x.device)
        need_w, need_b = ctx.needs_input_grad[2], bias is not None and ctx.needs_input_grad[3]
        direct = (need_w and weight.grad is not None and weight.grad.is_contiguous()
                  and (not need_b or bias.grad is not None))
        dW = weight.grad if direct else (torch.zeros_like(weight) if need_w else None)
        db = (bias.grad if direct else torch.zeros_like(bias)) if need_b else None
        _ext.call("mda_abf_bwd", dout, x, y, att, weight.detach().reshape(2, 2 * C).contiguous(),
                  dx, dy, dyup, part, dW, db, N, h, w, hy, wy, C, nb.value, 1)
        if direct:
            from ..parallel.grad_reducer import notify_grad
            notify_grad(weight, *([bias] if need_b else []))
            return dx, dy, None, None
        return dx, dy, dW, db


def _abf_native_ok(x, y, att_conv) -> bool:
    from ..ops.backend import hip_enabled_for
    if not (hip_enabled_for(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and y.dim() == 4):
        return False
    C = x.shape[1]
    G = C // 8
    conv = att_conv[0]
    return (C % 8 == 0 and 0 < G <= 64 and (G & (G - 1)) == 0 and y.shape[1] == C
            and conv.weight.shape == (2, 2 * C, 1, 1) and conv.weight.dtype == torch.float32
            and x.shape[0] == y.shape[0])


class ABF(nn.Module):
    def __init__(self, in_channel, mid_channel, out_channel, fuse):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(in_channel, mid_channel, kernel_size=1, bias=False),
                                   nn.BatchNorm2d(mid_channel))
        self.conv2 = nn.Sequential(nn.Conv2d(mid_channel, out_channel, kernel_size=3, stride=1,
                                             padding=1, bias=False),
                                   nn.BatchNorm2d(out_channel))
        if fuse:
            self.att_conv = nn.Sequential(nn.Conv2d(mid_channel * 2, 2, kernel_size=1), nn.Sigmoid())
        else:
            self.att_conv = None
        nn.init.kaiming_uniform_(self.conv1[0].weight, a=1)
        nn.init.kaiming_uniform_(self.conv2[0].weight, a=1)

    def forward(self, x, y=None, shape=None, out_shape=None):
        n, _, h, w = x.shape
        x = conv_bn_act(x, self.conv1[0], self.conv1[1], "none")[0]
        if self.att_conv is not None:
            if x.shape[-2:] == (shape, shape) and _abf_native_ok(x, y, self.att_conv):
                x = _ABFFuse.apply(x, y, self.att_conv[0].weight, self.att_conv[0].bias)
            else:
                y = F.interpolate(y, (shape, shape), mode="nearest")
                z = self.att_conv(torch.cat([x, y.to(x.dtype)], dim=1))
                x = x * z[:, 0].view(n, 1, h, w) + y * z[:, 1].view(n, 1, h, w)
        if x.shape[-1] != out_shape:
            x = F.interpolate(x, (out_shape, out_shape), mode="nearest")
        y = conv_bn_act(x, self.conv2[0], self.conv2[1], "none")[0]
        return y, x


class ReviewKD(Distiller):
    teacher_needs = ("preact", "pooled")

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.shapes = cfg.REVIEWKD.SHAPES
        self.out_shapes = cfg.REVIEWKD.OUT_SHAPES
        in_channels = cfg.REVIEWKD.IN_CHANNELS
        out_channels = cfg.REVIEWKD.OUT_CHANNELS
        self.ce_loss_weight = cfg.REVIEWKD.CE_WEIGHT
        self.reviewkd_loss_weight = cfg.REVIEWKD.REVIEWKD_WEIGHT
        self.warmup_epochs = cfg.REVIEWKD.WARMUP_EPOCHS
        self.stu_preact = cfg.REVIEWKD.STU_PREACT
        self.max_mid_channel = cfg.REVIEWKD.MAX_MID_CHANNEL
        mid_channel = min(self.max_mid_channel, in_channels[-1])
        abfs = [ABF(c, mid_channel, out_channels[i], i < len(in_channels) - 1)
                for i, c in enumerate(in_channels)]
        self.abfs = nn.ModuleList(abfs[::-1])

    def get_extra_parameters(self) -> int:
        return sum(p.numel() for p in self.abfs.parameters())

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, fs = self.student(image)
        _, ft = t_out.get()
        key = "preact_feats" if self.stu_preact else "feats"
        pooled_s = fs["pooled_feat"].reshape(fs["pooled_feat"].shape[0], -1, 1, 1)
        x = (list(fs[key][1:]) + [pooled_s])[::-1]
        results = []
        out, res = self.abfs[0](x[0], out_shape=self.out_shapes[0])
        results.append(out)
        for feat, abf, shape, out_shape in zip(x[1:], self.abfs[1:], self.shapes[1:],
                                               self.out_shapes[1:]):
            out, res = abf(feat, res, shape, out_shape)
            results.insert(0, out)
        pooled_t = ft["pooled_feat"].reshape(ft["pooled_feat"].shape[0], -1, 1, 1)
        t_feats = list(ft["preact_feats"][1:]) + [pooled_t]
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_kd = FL.hcl_loss_weighted(results, t_feats, self.reviewkd_loss_weight,
                                       kwargs.get("epoch"), self.warmup_epochs)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_kd}
