"""ReviewKD fused kernels (csrc/reviewkd.hip) vs fp32 PyTorch: HCL over every
level shape class (pyramid, adaptive overlapping bins, 1x1 pooled level)
with weight/warm-up, and the ABF attention fusion forward + all gradients."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import feat_losses as FL
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shapes", [
    [(16, 64, 32), (16, 128, 16), (16, 256, 8), (16, 256, 1)],   # CIFAR ReviewKD levels
    [(4, 64, 56), (4, 128, 28), (4, 256, 14), (4, 512, 7), (4, 512, 1)],  # ImageNet (7x7: overlapping bins)
    [(3, 24, 5), (3, 12, 3), (3, 8, 2)],
    [(2, 3, 64), (2, 6, 48), (2, 96, 9)],  # 1 / 2 / 32 channels per block
])
@pytest.mark.parametrize("epoch,warmup", [(None, 0.0), (0.5, 1.0)])
def test_hcl_fused(shapes, epoch, warmup):
    torch.manual_seed(0)
    fs = [_bf(torch.randn(n, c, h, h, device=DEV)) for n, c, h in shapes]
    ft = [_bf(torch.randn(n, c, h, h, device=DEV)) for n, c, h in shapes]
    ep = torch.tensor(epoch, device=DEV) if epoch is not None else None
    xs = [f.detach().clone().requires_grad_(True) for f in fs]
    with use_backend("hip"):
        assert FL.hcl_native_ok(xs, ft)
        loss = FL.hcl_loss_weighted(xs, ft, 5.0, ep, warmup)
    loss.backward()
    xr = [f.detach().float().requires_grad_(True) for f in fs]
    f = 5.0 * (min(epoch / warmup, 1.0) if epoch is not None and warmup > 0 else 1.0)
    ref = f * FL.hcl_loss(xr, [t.float() for t in ft])
    ref.backward()
    torch.testing.assert_close(loss, ref.detach(), rtol=2e-4, atol=1e-5)
    for a, b in zip(xs, xr):
        rel = ((a.grad.float() - b.grad).norm() / b.grad.norm()).item()
        assert rel < 1e-2, rel


@pytest.mark.parametrize("N,C,h,hy", [(8, 256, 8, 1), (8, 256, 16, 8), (4, 256, 32, 16),
                                      (2, 512, 14, 7), (4, 64, 8, 8)])
def test_abf_fuse(N, C, h, hy):
    from mdistiller_ddp_amd.distillers.ReviewKD import _ABFFuse
    torch.manual_seed(1)
    att = nn.Sequential(nn.Conv2d(2 * C, 2, kernel_size=1), nn.Sigmoid()).to(DEV)
    x = _bf(torch.randn(N, C, h, h, device=DEV))
    y = _bf(torch.randn(N, C, hy, hy, device=DEV))
    x1, y1 = x.clone().requires_grad_(True), y.clone().requires_grad_(True)
    out = _ABFFuse.apply(x1, y1, att[0].weight, att[0].bias)
    g = torch.randn(N, C, h, h, device=DEV).to(torch.bfloat16).float()
    out.float().backward(g)
    gw, gb = att[0].weight.grad.clone(), att[0].bias.grad.clone()
    att[0].weight.grad = None
    att[0].bias.grad = None
    x2, y2 = x.float().requires_grad_(True), y.float().requires_grad_(True)
    yu = F.interpolate(y2, (h, h), mode="nearest")
    z = att(torch.cat([x2, yu], dim=1))
    ref = x2 * z[:, 0:1] + yu * z[:, 1:2]
    ref.backward(g)

    def rel(a, b):
        return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()

    torch.testing.assert_close(out.float(), ref.detach(), atol=3e-2, rtol=2e-2)
    assert rel(x1.grad, x2.grad) < 1e-2
    assert rel(y1.grad, y2.grad) < 1e-2
    assert rel(gw, att[0].weight.grad) < 1e-2
    assert rel(gb, att[0].bias.grad) < 1e-2
