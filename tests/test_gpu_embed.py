"""CRD's Embed head on csrc/embed.hip (linear + l2 normalise, forward and
backward) vs the PyTorch fp32 composition of the reference (CRD.py:101-113)."""
import pytest
import torch

from mdistiller_ddp_amd.distillers.CRD import Embed
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,K,D", [(64, 256, 128), (32, 1024, 128), (7, 68, 40)])
def test_embed_matches_torch(N, K, D):
    torch.manual_seed(0)
    e = Embed(K, D).cuda()
    x = torch.randn(N, K, device="cuda", requires_grad=True)
    g = torch.randn(N, D, device="cuda")
    with use_backend("hip"):
        y = e(x)
    (y * g).sum().backward()
    dx, dw, db = x.grad.clone(), e.linear.weight.grad.clone(), e.linear.bias.grad.clone()
    x.grad = None
    e.zero_grad()
    with use_backend("torch"):
        yr = e(x)
    (yr * g).sum().backward()
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y, yr) < 1e-5
    assert rel(dx, x.grad) < 1e-4
    assert rel(dw, e.linear.weight.grad) < 1e-4
    assert rel(db, e.linear.bias.grad) < 1e-4
