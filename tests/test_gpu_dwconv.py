"""Depthwise 3x3 HIP kernels (csrc/dwconv.hip) vs fp32 PyTorch: folded-BN
inference path (teacher), training path (conv + BN + residual + act forward,
running stats, x / weight / gamma / beta / residual gradients)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_layers, hip_train
from mdistiller_ddp_amd.ops.backend import use_backend
from mdistiller_ddp_amd.ops import nn as mnn

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, C, H, stride
    (8, 32, 32, 1),
    (8, 96, 16, 2),
    (4, 60, 15, 1),     # ShuffleNetV1 widths (C % 8 != 0 -> 4-wide vectors)
    (4, 144, 8, 2),
    (2, 960, 7, 1),
    (3, 6, 9, 2),       # 2-wide vectors, odd sizes
    (2, 32, 112, 1),    # MobileNetV1 112^2 (LDS-tiled kernels: several row tiles)
    (2, 64, 112, 2),
    (2, 512, 14, 1),
    (2, 1024, 7, 1),
    (3, 40, 20, 2),     # 8-channel chunks
]


def _rel(a, b):
    return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act,with_res", [("relu", False), ("relu6", True), ("none", False)])
def test_dw_inference_folded_bn(shape, act, with_res):
    N, C, H, s = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(C, C, 3, s, 1, groups=C, bias=False).cuda().eval()
    bn = nn.BatchNorm2d(C).cuda().eval()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
    conv.weight.requires_grad_(False)
    bn.weight.requires_grad_(False)
    bn.bias.requires_grad_(False)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // s + 1
    res = torch.randn(N, C, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    with torch.no_grad(), use_backend("hip"):
        assert hip_layers.conv_supported(x, conv, bn)
        out, pre = mnn.conv_bn_act(x, conv, bn, act, res, want_preact=True)
        z = bn(conv(x.float()))
        if with_res:
            z = z + res.float()
        o = {"relu": F.relu, "relu6": F.relu6, "none": lambda t: t}[act](z)
    torch.testing.assert_close(pre.float(), z, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(out.float(), o, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("shape", [sh for sh in SHAPES if sh[1] % 8 == 0])
@pytest.mark.parametrize("act,with_res", [("relu", True), ("relu6", False), ("none", False)])
def test_dw_bn_act_train(shape, act, with_res):
    N, C, H, s = shape
    torch.manual_seed(1)
    conv = nn.Conv2d(C, C, 3, s, 1, groups=C, bias=False).cuda()
    bn = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // s + 1
    res = torch.randn(N, C, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    x1 = x.clone().requires_grad_(True)
    r1 = res.clone().requires_grad_(True) if with_res else None
    assert hip_train.train_supported(x1, conv, bn)
    out, pre = hip_train.conv_bn_act_train(x1, conv, bn, act, r1, True)
    g = torch.randn_like(out.float()).to(torch.bfloat16).float()
    gp = (torch.randn_like(out.float()) * 0.1).to(torch.bfloat16).float()
    torch.autograd.backward([out.float(), pre.float()], [g, gp])
    x2 = x.float().clone().requires_grad_(True)
    r2 = res.float().clone().requires_grad_(True) if with_res else None
    z = bn_r(conv_r(x2))
    if with_res:
        z = z + r2
    o = {"relu": F.relu, "relu6": F.relu6, "none": lambda t: t}[act](z)
    torch.autograd.backward([o, z], [g, gp])
    tol = 4e-2
    torch.testing.assert_close(out.float(), o, atol=tol, rtol=tol)
    torch.testing.assert_close(pre.float(), z, atol=tol, rtol=tol)
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, bn_r.running_var, atol=1e-2, rtol=1e-2)
    assert _rel(bn.weight.grad, bn_r.weight.grad) < 5e-2
    assert _rel(bn.bias.grad, bn_r.bias.grad) < 5e-2
    assert _rel(conv.weight.grad, conv_r.weight.grad) < 5e-2
    assert _rel(x1.grad, x2.grad) < 5e-2
    if with_res:
        assert _rel(r1.grad, r2.grad) < 5e-2


@pytest.mark.parametrize("shape", SHAPES)
def test_dw_dgrad_wgrad_exact_inputs(shape):
    from mdistiller_ddp_amd.ops import _ext
    N, C, H, s = shape
    torch.manual_seed(2)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, 1, 3, 3, device="cuda") * 0.3)
    Ho = (H + 2 - 3) // s + 1
    dy = torch.randn(N, C, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=s, padding=1, groups=C).backward(dy.float())
    wp = hip_train.dw_pack(w)
    dx = torch.empty_like(x)
    _ext.call("mda_dw_dgrad", dy, wp, dx, N, H, H, C, Ho, Ho, 3, 3, s, 1)
    nblk = hip_train._dw_wgrad_blocks(N, H, H, C, Ho, Ho, s)
    part = torch.empty(nblk * 9 * C, device="cuda")
    dw = torch.full_like(w, 1.0)
    _ext.call("mda_dw_wgrad", x, dy, part, dw, N, H, H, C, Ho, Ho, 3, 3, s, 1, nblk, 1)
    assert _rel(dx, xr.grad) < 1e-2
    assert _rel(dw - 1.0, wr.grad) < 1e-3
