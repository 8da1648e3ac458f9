"""MFMA implicit-GEMM conv (+folded BN, residual, activation) vs PyTorch fp32."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_layers

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, Cin, H, Cout, k, stride, pad
    (64, 3, 32, 32, 3, 1, 1),     # r32x4 stem (input padded to 8 channels)
    (8, 3, 64, 64, 7, 2, 3),      # ImageNet 7x7/s2 stem (padded)
    (64, 32, 32, 64, 3, 1, 1),    # layer1 first conv
    (64, 64, 32, 64, 3, 1, 1),
    (64, 64, 32, 128, 3, 2, 1),   # stride-2 transition
    (64, 128, 16, 128, 3, 1, 1),
    (64, 128, 16, 256, 3, 2, 1),
    (64, 256, 8, 256, 3, 1, 1),
    (64, 64, 32, 128, 1, 2, 0),   # 1x1 shortcut
    (64, 64, 32, 128, 3, 1, 1),   # 128x128 tile
    (8, 16, 32, 16, 3, 1, 1),     # resnet20 (vec8 loader)
    (5, 24, 15, 40, 3, 2, 1),     # odd everything
    (3, 96, 7, 100, 1, 1, 0),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act", ["relu", "none"])
@pytest.mark.parametrize("with_res", [False, True])
def test_conv_bn_act_inference(shape, act, with_res):
    N, Cin, H, Cout, k, s, p = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda()
    with torch.no_grad():
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn.eval()
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    with torch.no_grad():
        ref = bn(conv(x.float()))
        if res is not None:
            ref = ref + res.float()
        pre_ref = ref
        ref = F.relu(ref) if act == "relu" else ref
        assert hip_layers.conv_supported(x, conv, bn)
        y, pre = hip_layers.conv_bn_act(x, conv, bn, act, res, True)
    assert y.dtype == torch.bfloat16 and y.shape == ref.shape
    tol = 3e-2 * max(1.0, ref.abs().max().item() / 4)
    torch.testing.assert_close(y.float(), ref, atol=tol, rtol=2e-2)
    torch.testing.assert_close(pre.float(), pre_ref, atol=tol, rtol=2e-2)


def test_teacher_forward_matches_torch():
    from mdistiller_ddp_amd.models.cifar import resnet32x4
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(0)
    m = resnet32x4(num_classes=100).cuda().eval()
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        ref, _ = m(x)
        with torch.autocast("cuda", dtype=torch.bfloat16), use_backend("hip"):
            out, feats = m(x)
    rel = (out.float() - ref).norm() / ref.norm()
    assert rel < 3e-2, rel


DGRAD_SHAPES = [
    # N, Cin, H, Cout, k, stride, pad   (dgrad: dx of conv(x))
    (4, 64, 32, 128, 3, 2, 1),    # parity classes 1/2/2/4 taps
    (2, 64, 56, 128, 3, 2, 1),    # ImageNet layer2 transition
    (3, 32, 15, 64, 3, 2, 1),     # odd extent
    (2, 64, 32, 128, 1, 2, 0),    # 1x1 / s2: three classes have no taps
    (2, 8, 30, 64, 7, 2, 3),      # 7x7 / s2 (stem-like)
    (2, 64, 16, 64, 3, 1, 1),     # stride 1 (halo)
    (8, 64, 8, 64, 3, 1, 1),      # 8x8 maps: 3 images per 256-pixel block, partial last block
    (4, 32, 32, 64, 3, 1, 1),     # dgrad with 32 output channels (BN = 32 tiles)
    (2, 64, 56, 64, 3, 1, 1),     # stride 1, width 56 (halo, 112-pixel blocks)
    (2, 128, 28, 128, 3, 1, 1),   # width 28, two channel chunks
    (2, 128, 14, 128, 3, 1, 1),   # width 14 (98-pixel blocks)
    (4, 256, 7, 256, 3, 1, 1),    # 7x7 maps, two images per block
]


@pytest.mark.parametrize("shape", DGRAD_SHAPES)
def test_conv_dgrad_matches_autograd(shape):
    from mdistiller_ddp_amd.ops import hip_train
    N, Cin, H, Cout, k, s, p = shape
    torch.manual_seed(0)
    w = torch.randn(Cout, Cin, k, k, device="cuda") / (Cin * k * k) ** 0.5
    x = torch.randn(N, Cin, H, H, device="cuda").requires_grad_(True)
    y = F.conv2d(x, w.to(torch.bfloat16).float(), stride=s, padding=p)
    g = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(g)
    dx = hip_train.conv_dgrad(g.to(torch.bfloat16), w, x.shape, s, p)
    torch.testing.assert_close(dx.float(), x.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("shape", [(2, 64, 56, 64, 3, 1, 1), (4, 64, 32, 32, 3, 1, 1),
                                   (5, 64, 8, 64, 3, 1, 1), (2, 128, 28, 128, 3, 1, 1),
                                   (2, 256, 14, 256, 3, 1, 1), (4, 512, 7, 512, 3, 1, 1)])
def test_conv_forward_imagenet_widths(shape):
    """Halo kernel with blocks of whole rows that do not fill 128 pixels."""
    N, Cin, H, Cout, k, s, p = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda().eval()
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.float(), conv.weight.to(torch.bfloat16).float(), stride=s, padding=p)
    with torch.no_grad():
        out, _ = hip_layers.conv_bn_act(x, conv, None, "none", None, False)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
