"""Streaming 1x1 conv (csrc/conv1x1.hip: transposed MFMA, resident weights,
stores straight from the accumulators) vs PyTorch fp32: inference epilogue
(folded BN, residual, activation, pre-activation), the training forward with
BN batch statistics, and the stride-1 dgrad.  Shapes cover K = 32 / 64 / 96 / 128 / 192 /
256, 64 / 128 / 256-channel slices (and half-live 32-channel ones), stride 2 and an M tail."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_layers, hip_train

pytestmark = pytest.mark.gpu

SHAPES = [  # N, Cin, H, Cout, stride
    (16, 64, 56, 256, 1),   # bottleneck expand (CI = 4)
    (16, 256, 56, 64, 1),   # bottleneck reduce (K = 256, CI = 1)
    (8, 128, 28, 512, 1),   # K = 128 (CI = 2)
    (8, 192, 48, 128, 1),   # K = 192
    (3, 64, 99, 128, 1),    # M = 29403: tail tile
    (16, 128, 56, 256, 2),  # stride-2 projection shortcut
    (8, 32, 112, 64, 1),    # K = 32 on 64-padded weight rows (MobileNetV1's first pointwise)
    (8, 96, 40, 128, 1),    # K = 96 (Kp = 128)
    (8, 64, 40, 96, 1),     # dgrad K = 96 (LOAD_DGRAD_VEC8 mode reaches the stream kernel)
    (8, 64, 48, 32, 1),     # Cout = 32: one half-live 64-channel slice
    (8, 192, 32, 96, 1),    # Cout = 96: a full and a half-live slice
    (16, 64, 32, 160, 2),   # Cout = 160, stride 2
]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act,with_res", [("relu", True), ("none", False)])
def test_stream_inference(shape, act, with_res):
    N, Cin, H, Cout, s = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, 1, s, 0, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda().eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H - 1) // s + 1
    res = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) if with_res else None
    with torch.no_grad():
        out, pre = hip_layers.conv_bn_act(x, conv, bn, act, res, True)
        ref = bn(conv(x.float()))
        if res is not None:
            ref = ref + res.float()
        ref_out = F.relu(ref) if act == "relu" else ref
    assert _rel(out, ref_out) < 1e-2
    assert pre is not None and _rel(pre, ref) < 1e-2


@pytest.mark.parametrize("shape", SHAPES)
def test_stream_train_forward_stats_and_dgrad(shape):
    N, Cin, H, Cout, s = shape
    torch.manual_seed(1)
    conv = nn.Conv2d(Cin, Cout, 1, s, 0, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda().train()
    ref_conv, ref_bn = nn.Conv2d(Cin, Cout, 1, s, 0, bias=False).cuda(), nn.BatchNorm2d(Cout).cuda().train()
    ref_conv.load_state_dict(conv.state_dict())
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xx = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out, _ = hip_train.conv_bn_act_train(xx, conv, bn, "relu", None, False)
    xr = x.float().clone().requires_grad_(True)
    ref = F.relu(ref_bn(ref_conv(xr)))
    assert _rel(out, ref) < 2e-2
    assert _rel(bn.running_mean, ref_bn.running_mean) < 1e-2
    assert _rel(bn.running_var, ref_bn.running_var) < 1e-2
    g = torch.randn_like(ref)
    (out.float() * g).sum().backward()
    (ref * g).sum().backward()
    # (bf16 BN backward: dy is rounded before the dgrad; the pure dgrad is
    # held to 1e-2 below)
    assert _rel(xx.grad, xr.grad) < 5e-2
    assert _rel(conv.weight.grad, ref_conv.weight.grad) < 5e-2


@pytest.mark.parametrize("shape", [(16, 256, 56, 64), (8, 128, 28, 256), (3, 64, 99, 128),
                                   (8, 64, 40, 96), (8, 64, 112, 32), (64, 32, 32, 64),
                                   (16, 96, 32, 64)])
def test_stream_dgrad(shape):
    """dx = dgrad(dy) of a stride-1 1x1 conv (the stream kernel with W^T)."""
    N, Cin, H, Cout = shape
    torch.manual_seed(2)
    w = torch.randn(Cout, Cin, 1, 1, device="cuda") * 0.1
    dy = torch.randn(N, Cout, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dx = hip_train.conv_dgrad(dy, w, (N, Cin, H, H), 1, 0)
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w, dy.float(), 1, 0)
    assert _rel(dx, ref) < 1e-2
