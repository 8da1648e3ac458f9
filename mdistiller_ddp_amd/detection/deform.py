"""Deformable convolution (DCN v1) and modulated deformable convolution (DCN v2).

The detection ResNet's ``DeformBottleneckBlock`` (reference
``detection/model/backbone/resnet.py:223-336``) puts one of these in the 3x3
slot, fed by a plain 3x3 conv that predicts the per-tap offsets (18 channels
per deformable group; 27 with the DCN-v2 modulation mask).  The reference
takes the ops from Detectron2's CUDA extension; here they are written as a
bilinear gather (``im2col`` at fractional positions) followed by one grouped
GEMM, so autograd provides the input, offset, mask and weight gradients and
the GEMM runs on hipBLASLt.

Layout conventions (Detectron2 / mmcv): ``offset`` is
``[N, dg * KH * KW * 2, Ho, Wo]`` with, per deformable group and tap
``k = kh * KW + kw``, channel ``2k`` the row (y) offset and ``2k + 1`` the
column (x) offset; ``mask`` is ``[N, dg * KH * KW, Ho, Wo]``.  A sample that
falls outside the image contributes zero (the corners outside are dropped,
exactly the reference's bilinear rule).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.nn.modules.utils import _pair


def _bilinear_gather(x, py, px):
    """x: [N, G, Cg, H, W]; py, px: [N, G, P] fractional positions ->
    [N, G, Cg, P] bilinear samples with zero outside the image."""
    N, G, Cg, H, W = x.shape
    P = py.shape[-1]
    flat = x.reshape(N, G, Cg, H * W)
    y0 = torch.floor(py)
    x0 = torch.floor(px)
    ly, lx = py - y0, px - x0
    y0 = y0.long()
    x0 = x0.long()
    out = None
    for dy, wy in ((0, 1 - ly), (1, ly)):
        for dx, wx in ((0, 1 - lx), (1, lx)):
            yy, xx = y0 + dy, x0 + dx
            ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            idx = (yy.clamp(0, H - 1) * W + xx.clamp(0, W - 1))
            v = flat.gather(3, idx.view(N, G, 1, P).expand(N, G, Cg, P))
            w = (wy * wx * ok.to(wy.dtype)).view(N, G, 1, P)
            out = v * w if out is None else out + v * w
    return out


class _DeformConvFn(torch.autograd.Function):
    """Deformable conv on the HIP sampling kernels (ops/csrc/deform.hip): the
    bilinear gather (and its scatter / coordinate-gradient backward) native,
    the three GEMMs (out, dW, dcols) batched on hipBLASLt."""

    @staticmethod
    def forward(ctx, x, offset, mask, weight, bias, meta):
        from ..ops import _ext
        (sh, sw), (ph, pw), (dh, dw), groups, dg = meta
        x = x.contiguous()
        dt = x.dtype
        off = offset.to(dt).contiguous()
        m = mask.to(dt).contiguous() if mask is not None else None
        N, C, H, W = x.shape
        Cout, Cg, KH, KW = weight.shape
        K = KH * KW
        Ho = (H + 2 * ph - (dh * (KH - 1) + 1)) // sh + 1
        Wo = (W + 2 * pw - (dw * (KW - 1) + 1)) // sw + 1
        L = Ho * Wo
        geom = torch.tensor([N, C, H, W, Ho, Wo, KH, KW, sh, sw, ph, pw, dh, dw, dg], dtype=torch.int64)
        cols = torch.empty(N, C * K, L, dtype=dt, device=x.device)
        code = 0 if dt == torch.float32 else 1
        _ext.call("mda_deform_im2col", code, x, off, m, cols, geom)
        w = weight.to(dt).reshape(groups, Cout // groups, Cg * K)
        out = torch.matmul(w, cols.view(N, groups, Cg * K, L)).reshape(N, Cout, Ho, Wo)
        if bias is not None:
            out = out + bias.to(dt).view(1, Cout, 1, 1)
        ctx.save_for_backward(x, off, m, weight, cols)
        ctx.meta = (geom, groups, code, Ho, Wo, offset.dtype, mask.dtype if mask is not None else None,
                    bias is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..ops import _ext
        x, off, m, weight, cols = ctx.saved_tensors
        geom, groups, code, Ho, Wo, off_dt, mask_dt, has_b = ctx.meta
        N, C, H, W = x.shape
        Cout, Cg, KH, KW = weight.shape
        K, L = KH * KW, Ho * Wo
        dt = x.dtype
        d = dout.to(dt).contiguous().view(N, groups, Cout // groups, L)
        colsg = cols.view(N, groups, Cg * K, L)
        dw = torch.matmul(d, colsg.transpose(-1, -2)).sum(0).reshape(weight.shape).to(weight.dtype)
        w = weight.to(dt).reshape(groups, Cout // groups, Cg * K)
        dcols = torch.matmul(w.transpose(-1, -2), d).reshape(N, C * K, L).contiguous()
        dx = torch.zeros(N, C, H, W, dtype=torch.float32, device=x.device)
        doff = torch.empty_like(off)
        dmask = torch.empty_like(m) if m is not None else None
        _ext.call("mda_deform_col2im", code, dcols, x, off, m, dx, doff, dmask, geom)
        db = d.float().sum((0, 3)).reshape(Cout).to(weight.dtype) if has_b else None
        return (dx.to(dt), doff.to(off_dt), dmask.to(mask_dt) if dmask is not None else None, dw,
                db, None)


def _native_ok(x, offset, weight):
    from ..ops.backend import hip_enabled_for
    return (x.dim() == 4 and hip_enabled_for(x) and x.dtype in (torch.float32, torch.bfloat16)
            and weight.dtype in (torch.float32, torch.bfloat16))


def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1, mask=None):
    """Deformable 2-D convolution (``mask`` given: modulated, DCN v2).  On the
    GPU the sampling runs on the HIP kernels (:class:`_DeformConvFn`), else as
    the PyTorch gather below."""
    if _native_ok(x, offset, weight):
        N, C, H, W = x.shape
        Cout, Cg, KH, KW = weight.shape
        if C % deformable_groups or C != Cg * groups or Cout % groups:
            raise ValueError(f"deform_conv2d: channels {C} / groups {groups} / deformable groups "
                             f"{deformable_groups}")
        meta = (_pair(stride), _pair(padding), _pair(dilation), groups, deformable_groups)
        return _DeformConvFn.apply(x, offset, mask, weight, bias, meta)
    return _deform_conv2d_torch(x, offset, weight, bias, stride, padding, dilation, groups,
                                deformable_groups, mask)


def _deform_conv2d_torch(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                         deformable_groups=1, mask=None):
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    N, C, H, W = x.shape
    Cout, Cg, KH, KW = weight.shape
    K = KH * KW
    dg = deformable_groups
    if C % dg or C != Cg * groups or Cout % groups:
        raise ValueError(f"deform_conv2d: channels {C} / groups {groups} / deformable groups {dg}")
    Ho = (H + 2 * ph - (dh * (KH - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (KW - 1) + 1)) // sw + 1
    if offset.shape != (N, dg * K * 2, Ho, Wo):
        raise ValueError(f"deform_conv2d: offset shape {tuple(offset.shape)} != {(N, dg * K * 2, Ho, Wo)}")
    dt = x.dtype
    off = offset.to(dt).view(N, dg, K, 2, Ho, Wo)
    dev = x.device
    ky = (torch.arange(KH, device=dev, dtype=dt) * dh).repeat_interleave(KW)      # [K]
    kx = (torch.arange(KW, device=dev, dtype=dt) * dw).repeat(KH)                 # [K]
    oy = torch.arange(Ho, device=dev, dtype=dt) * sh - ph                          # [Ho]
    ox = torch.arange(Wo, device=dev, dtype=dt) * sw - pw                          # [Wo]
    py = ky.view(1, 1, K, 1, 1) + oy.view(1, 1, 1, Ho, 1) + off[:, :, :, 0]       # [N, dg, K, Ho, Wo]
    px = kx.view(1, 1, K, 1, 1) + ox.view(1, 1, 1, 1, Wo) + off[:, :, :, 1]
    L = Ho * Wo
    cols = _bilinear_gather(x.view(N, dg, C // dg, H, W), py.reshape(N, dg, K * L),
                            px.reshape(N, dg, K * L))                               # [N, dg, C/dg, K*L]
    cols = cols.view(N, dg, C // dg, K, L)
    if mask is not None:
        if mask.shape != (N, dg * K, Ho, Wo):
            raise ValueError(f"deform_conv2d: mask shape {tuple(mask.shape)} != {(N, dg * K, Ho, Wo)}")
        cols = cols * mask.to(dt).view(N, dg, 1, K, L)
    cols = cols.reshape(N, groups, Cg * K, L)                                       # channel-major, tap-minor
    w = weight.to(dt).view(groups, Cout // groups, Cg * K)
    out = torch.einsum("gok,ngkl->ngol", w, cols).reshape(N, Cout, Ho, Wo)
    if bias is not None:
        out = out + bias.to(dt).view(1, Cout, 1, 1)
    return out


class _DeformBase(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, deformable_groups=1, bias=False, norm=None, activation=None):
        super().__init__()
        if in_channels % groups or out_channels % groups:
            raise ValueError("channels must be divisible by groups")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride, self.padding, self.dilation = _pair(stride), _pair(padding), _pair(dilation)
        self.groups, self.deformable_groups = groups, deformable_groups
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels // groups, *self.kernel_size))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
        self.norm, self.activation = norm, activation
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def _post(self, out):
        if self.norm is not None:
            out = self.norm(out)
        if self.activation is not None:
            out = self.activation(out)
        return out

    def extra_repr(self):
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, dilation={self.dilation}, "
                f"groups={self.groups}, deformable_groups={self.deformable_groups}, bias={self.bias is not None}")


class DeformConv(_DeformBase):
    """DCN v1: ``forward(x, offset)``."""

    def forward(self, x, offset):
        out = deform_conv2d(x, offset, self.weight, self.bias, self.stride, self.padding,
                            self.dilation, self.groups, self.deformable_groups)
        return self._post(out)


class ModulatedDeformConv(_DeformBase):
    """DCN v2: ``forward(x, offset, mask)`` with ``mask`` in [0, 1]."""

    def forward(self, x, offset, mask):
        out = deform_conv2d(x, offset, self.weight, self.bias, self.stride, self.padding,
                            self.dilation, self.groups, self.deformable_groups, mask=mask)
        return self._post(out)
