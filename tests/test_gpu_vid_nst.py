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
    assert rel(fs1.grad, fs2.grad) < 5e-2
    for (n, p), (_, q) in zip(reg.named_parameters(), reg_r.named_parameters()):
        assert rel(p.grad, q.grad) < 5e-2, n
