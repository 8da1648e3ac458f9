"""Shared distiller building blocks (reference `distillers/_common.py:6-49`)."""
from __future__ import annotations

import torch
import torch.nn as nn

from ..models._base import Lambda  # noqa: F401  (re-export, reference API)
from ..ops.nn import conv_bn_act


class ConvReg(nn.Module):
    """Convolutional regressor mapping a student feature map onto a teacher's.

    Picks the layer from the spatial ratio (reference `_common.py:6-30`):
    student 2x larger -> 3x3 stride-2 conv; 2x smaller -> 4x4 stride-2
    transposed conv; otherwise a valid conv of size (1 + dH, 1 + dW).
    Followed by BN (+ReLU).  The conv+BN(+ReLU) runs through the fused op.
    """

    def __init__(self, s_shape, t_shape, use_relu: bool = True):
        super().__init__()
        self.use_relu = use_relu
        _, s_C, s_H, s_W = s_shape
        _, t_C, t_H, t_W = t_shape
        if s_H == 2 * t_H:
            self.conv = nn.Conv2d(s_C, t_C, kernel_size=3, stride=2, padding=1)
        elif s_H * 2 == t_H:
            self.conv = nn.ConvTranspose2d(s_C, t_C, kernel_size=4, stride=2, padding=1)
        elif s_H >= t_H:
            self.conv = nn.Conv2d(s_C, t_C, kernel_size=(1 + s_H - t_H, 1 + s_W - t_W))
        else:
            raise NotImplementedError(f"student size {s_H}, teacher size {t_H}")
        self.bn = nn.BatchNorm2d(t_C)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        act = "relu" if self.use_relu else "none"
        if isinstance(self.conv, nn.Conv2d):
            return conv_bn_act(x, self.conv, self.bn, act)[0]
        y = self.bn(self.conv(x))
        return torch.relu(y) if self.use_relu else y


@torch.no_grad()
def get_feat_shapes(student, teacher, input_size):
    """Feature shapes from a dry batch-1 CPU forward (eval mode, so the dry
    run does not touch BN running statistics as the reference's does)."""
    data = torch.randn(1, 3, *input_size)
    out = []
    for m in (student, teacher):
        if m is None:
            out.append(None)
            continue
        was = m.training
        dev = next(m.parameters()).device
        m.eval()
        feats = m(data.to(dev))[1]
        m.train(was)
        out.append([f.shape for f in feats["feats"]])
    return out[0], out[1]


def pool_to_match(f_s, f_t):
    """Adaptive-avg-pool the larger map to the smaller's size (AT/NST)."""
    s_H, t_H = f_s.shape[2], f_t.shape[2]
    if s_H > t_H:
        f_s = nn.functional.adaptive_avg_pool2d(f_s, (t_H, t_H))
    elif s_H < t_H:
        f_t = nn.functional.adaptive_avg_pool2d(f_t, (s_H, s_H))
    return f_s, f_t
