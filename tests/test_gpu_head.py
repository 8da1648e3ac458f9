"""HIP head/metrics kernels vs fp32 PyTorch references: fused global-avg-pool
+ Linear (forward, input/weight/bias gradients, flat-grad accumulation),
on-device metric update, DKD with the in-kernel warm-up factor."""
import pytest
import torch
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import losses as L
from mdistiller_ddp_amd.ops import nn as mnn
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,C,HW,J", [(64, 256, 8, 100), (5, 64, 8, 10), (16, 512, 7, 1000), (3, 48, 4, 7),
                                     (64, 2048, 7, 1000), (33, 1024, 7, 1000)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pool_linear(N, C, HW, J, dtype):
    torch.manual_seed(0)
    fc = torch.nn.Linear(C, J).to(DEV)
    x = torch.randn(N, C, HW, HW, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    avg_r = F.avg_pool2d(xr, HW).flatten(1)
    out_r = F.linear(avg_r, fc.weight.detach(), fc.bias.detach())
    gl = torch.randn(N, J, device=DEV)
    gp = torch.randn(N, C, device=DEV)
    (out_r * gl).sum().add_((avg_r * gp).sum()).backward()
    gw_r, gb_r = torch.autograd.grad((F.linear(avg_r.detach(), fc.weight, fc.bias) * gl).sum(),
                                     (fc.weight, fc.bias))
    xh = x.detach().clone().requires_grad_(True)
    with use_backend("hip"):
        assert mnn._pool_fc_native(xh, fc, HW)
        avg, out = mnn.pool_linear(xh, fc, HW)
    assert out.dtype == dtype and avg.dtype == dtype
    (out.float() * gl).sum().add_((avg.float() * gp).sum()).backward()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(avg.float(), avg_r.detach(), atol=tol, rtol=tol)
    torch.testing.assert_close(out.float(), out_r.detach(), atol=tol * 4, rtol=tol)
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=tol, rtol=tol)
    torch.testing.assert_close(fc.weight.grad, gw_r, atol=tol * 8, rtol=tol)
    torch.testing.assert_close(fc.bias.grad, gb_r, atol=tol * 8, rtol=tol)


@pytest.mark.parametrize("C,J", [(64, 10), (512, 300)])  # fused / tiled backward
def test_pool_linear_accumulates_into_bound_grad(C, J):
    torch.manual_seed(1)
    fc = torch.nn.Linear(C, J).to(DEV)
    fc.weight.grad = torch.ones_like(fc.weight)
    fc.bias.grad = torch.ones_like(fc.bias)
    x = torch.randn(4, C, 8, 8, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with use_backend("hip"):
        _, out = mnn.pool_linear(x, fc, 8)
    out.float().sum().backward()
    avg = F.avg_pool2d(x.float(), 8).flatten(1)
    torch.testing.assert_close(fc.bias.grad, torch.ones(J, device=DEV) + 4, atol=1e-5, rtol=0)
    torch.testing.assert_close(fc.weight.grad, 1 + avg.bfloat16().float().sum(0).expand(J, C),
                               atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_meters_kernel(dtype, ties):
    from mdistiller_ddp_amd.engine.step import DeviceMeters
    torch.manual_seed(2)
    keys = ["loss_ce", "loss_kd"]
    m_h, m_r = DeviceMeters(DEV, keys), DeviceMeters(DEV, keys)
    for _ in range(3):
        preds = torch.randn(64, 100, device=DEV).to(dtype)
        if ties:  # heavy ties with the target logit: stable-order rank, not a free hit
            preds = torch.randint(0, 3, (64, 100), device=DEV).to(dtype)
        target = torch.randint(0, 100, (64,), device=DEV)
        losses = {"loss_ce": torch.rand((), device=DEV), "loss_kd": torch.rand((), device=DEV)}
        with use_backend("hip"):
            assert m_h._native(preds, losses)
            m_h.update(preds, target, losses)
        with use_backend("torch"):
            m_r.update(preds, target, losses)
    torch.testing.assert_close(m_h.buf, m_r.buf, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("epoch,warmup", [(1.0, 20.0), (7.5, 5.0), (3.0, 0.0)])
def test_dkd_warmup_in_kernel(epoch, warmup):
    torch.manual_seed(3)
    s = (torch.randn(32, 100, device=DEV) * 3).requires_grad_(True)
    t = torch.randn(32, 100, device=DEV) * 3
    y = torch.randint(0, 100, (32,), device=DEV)
    ep = torch.tensor(epoch, device=DEV)
    with use_backend("hip"):
        ce, kd = L.ce_dkd(s, t, y, 1.0, 1.0, 8.0, 4.0, epoch=ep, warmup=warmup)
    g, = torch.autograd.grad(kd, s)
    f = min(epoch / warmup, 1.0) if warmup > 0 else 1.0
    s2 = s.detach().clone().requires_grad_(True)
    kd_r = f * L.dkd_loss_ref(s2, t, y, 1.0, 8.0, 4.0)
    g_r, = torch.autograd.grad(kd_r, s2)
    torch.testing.assert_close(kd, kd_r, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(g, g_r, atol=1e-5, rtol=1e-4)
