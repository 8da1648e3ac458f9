"""Native VID (csrc/feat.hip mda_vid_loss / mda_vid_bwd + three native 1x1
conv launches) vs the fp32 PyTorch formulation of the reference
(`distillers/VID.py:16-30`): loss, regressor / log-scale / student-feature
gradients."""
import copy
import math

import pytest
import torch
import torch.nn as nn

from mdistiller_ddp_amd.ops import feat_losses as FL
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu


def _reg(s, t):
    return nn.Sequential(nn.Conv2d(s, t, 1, bias=False), nn.ReLU(), nn.Conv2d(t, t, 1, bias=False),
                         nn.ReLU(), nn.Conv2d(t, t, 1, bias=False)).cuda()


@pytest.mark.parametrize("N,Cs,Ct,H", [(64, 64, 64, 32), (64, 128, 128, 16), (64, 256, 256, 8),
                                       (16, 64, 128, 16)])
def test_vid_native_matches_fp32(N, Cs, Ct, H):
    torch.manual_seed(0)
    reg = _reg(Cs, Ct)
    reg_r = copy.deepcopy(reg)
    init = math.log(math.exp(5.0 - 1e-5) - 1.0)
    ls = nn.Parameter(init * torch.ones(Ct, device="cuda") + 0.1 * torch.randn(Ct, device="cuda"))
    ls_r = nn.Parameter(ls.detach().clone())
    fs = torch.randn(N, Cs, H, H, device="cuda").relu().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ft = torch.randn(N, Ct, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    fs1 = fs.clone().requires_grad_(True)
    with use_backend("hip"):
        assert FL._vid_native_ok(reg, fs1, ft)
        loss = FL.vid_loss(reg, ls, fs1, ft, 1e-5)
    (3.0 * loss).backward()
    fs2 = fs.float().clone().requires_grad_(True)
    with use_backend("torch"):
        loss_r = FL.vid_loss(reg_r, ls_r, fs2, ft.float(), 1e-5)
    (3.0 * loss_r).backward()
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()  # noqa: E731
    assert abs(loss.item() - loss_r.item()) <= 1e-2 * abs(loss_r.item()) + 1e-4
    assert rel(ls.grad, ls_r.grad) < 2e-2
    assert rel(fs1.grad, fs2.grad) < 1e-1  # three bf16 dgrads with ReLU masks
    for (n, p), (_, q) in zip(reg.named_parameters(), reg_r.named_parameters()):
        assert rel(p.grad, q.grad) < 5e-2, n


@pytest.mark.parametrize("N,C,H", [(64, 64, 32), (64, 128, 16), (64, 256, 8)])
def test_nst_gram_matches_fp32(N, C, H):
    """GPU NST (one batched Gram per stage, closed-form backward) vs the fp32
    broadcast formulation on bf16 feature maps."""
    torch.manual_seed(1)
    fs = torch.randn(N, C, H, H, device="cuda").relu().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ft = torch.randn(N, C, H, H, device="cuda").relu().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = fs.clone().requires_grad_(True)
    with use_backend("hip"):
        loss = FL.nst_loss([a], [ft])
    loss.backward()
    b = fs.float().clone().requires_grad_(True)
    with use_backend("torch"):
        loss_r = FL.nst_loss([b], [ft.float()])
    loss_r.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_r.item()) <= 1e-3 * abs(loss_r.item()) + 1e-5
    assert ((a.grad.float() - b.grad).norm() / b.grad.norm()).item() < 2e-2


@pytest.mark.parametrize("k", [1, 3])
def test_convreg_bias_native_matches_fp32(k):
    """FitNet's ConvReg (conv WITH bias -> training BN -> ReLU,
    `distillers/_common.py:6-30`) on the native path: the conv runs without
    its bias (BN removes the shift; d bias = sum dy = 0) and the running mean
    takes it -- outputs, running stats and all gradients vs fp32 PyTorch."""
    from mdistiller_ddp_amd.distillers._common import ConvReg
    from mdistiller_ddp_amd.ops import hip_train
    torch.manual_seed(3)
    m = ConvReg((1, 64, 16 + k - 1, 16 + k - 1), (1, 128, 16, 16)).cuda()
    with torch.no_grad():
        m.conv.bias.uniform_(-1, 1)
    m_r = copy.deepcopy(m)
    x = torch.randn(32, 64, 16 + k - 1, 16 + k - 1, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    with use_backend("hip"):
        assert hip_train.train_supported(x1, m.conv, m.bn)
        out = m(x1)
    g = torch.randn_like(out.float())
    (out.float() * g).sum().backward()
    x2 = x.float().clone().requires_grad_(True)
    with use_backend("torch"):
        out_r = m_r(x2)
    (out_r * g).sum().backward()
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()  # noqa: E731
    assert rel(out, out_r) < 2e-2
    torch.testing.assert_close(m.bn.running_mean, m_r.bn.running_mean, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(m.bn.running_var, m_r.bn.running_var, atol=2e-2, rtol=2e-2)
    assert rel(x1.grad, x2.grad) < 5e-2
    assert rel(m.conv.weight.grad, m_r.conv.weight.grad) < 5e-2
    assert m.conv.bias.grad.abs().max().item() == 0.0
    assert m_r.conv.bias.grad.abs().max().item() < 1e-3 * m_r.conv.weight.grad.abs().max().item() + 1e-5
    assert rel(m.bn.weight.grad, m_r.bn.weight.grad) < 5e-2


@pytest.mark.parametrize("N,C,H", [(64, 256, 8), (64, 128, 16), (8, 64, 32)])
def test_fitnet_hint_mse_native_matches_fp32(N, C, H):
    """FitNet's hint loss (csrc/feat.hip mda_ofd_loss, no margin) vs
    weight * F.mse_loss in fp32 (reference `distillers/FitNet.py:41-43`)."""
    from mdistiller_ddp_amd.distillers.FitNet import hint_loss
    torch.manual_seed(0)
    fs = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ft = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a = fs.clone().requires_grad_(True)
    with use_backend("hip"):
        loss = hint_loss(a, ft, 100.0)
    (2.0 * loss).backward()
    b = fs.float().clone().requires_grad_(True)
    ref = 100.0 * torch.nn.functional.mse_loss(b, ft.float())
    (2.0 * ref).backward()
    assert loss.grad_fn is not None and "HintMSE" in type(loss.grad_fn).__name__
    torch.testing.assert_close(loss.float(), ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(a.grad.float(), b.grad, rtol=1e-2, atol=1e-6)
