"""Deformable conv on the HIP sampling kernels (ops/csrc/deform.hip) vs the
PyTorch gather composition (detection/deform.py), fp32: outputs and the
gradients of the input, offsets, modulation mask, weight and bias."""
import pytest
import torch

from mdistiller_ddp_amd.detection.deform import deform_conv2d
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu

CASES = [  # N, C, H, Cout, stride, pad, dil, groups, dg, modulated
    (2, 16, 12, 24, 1, 1, 1, 1, 1, True),
    (2, 16, 12, 24, 2, 1, 1, 1, 2, False),
    (1, 32, 9, 32, 1, 2, 2, 2, 4, True),
    (3, 8, 7, 8, 1, 1, 1, 1, 1, False),
]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("case", CASES)
def test_deform_conv_matches_torch(case):
    N, C, H, Co, s, p, d, g, dg, mod = case
    torch.manual_seed(0)
    Ho = (H + 2 * p - (d * 2 + 1)) // s + 1
    x = torch.randn(N, C, H, H, device="cuda")
    off = (torch.rand(N, dg * 18, Ho, Ho, device="cuda") - 0.5) * 6  # many samples outside
    m = torch.rand(N, dg * 9, Ho, Ho, device="cuda") if mod else None
    w = torch.randn(Co, C // g, 3, 3, device="cuda") * 0.1
    b = torch.randn(Co, device="cuda")
    gy = torch.randn(N, Co, Ho, Ho, device="cuda")
    outs = []
    # reference: the PyTorch gather composition in float64 on the CPU (this
    # ROCm build's GPU kernels are not trusted as a reference, see
    # profiles/r4_rocm_avgpool_cl_bug.md)
    for dev, dt in (("cuda", torch.float32), ("cpu", torch.float64)):
        leaves = [t.to(dev, dt).clone().requires_grad_(True) for t in (x, off, w, b)]
        mm = m.to(dev, dt).clone().requires_grad_(True) if m is not None else None
        with use_backend("hip" if dev == "cuda" else "torch"):
            y = deform_conv2d(leaves[0], leaves[1], leaves[2], leaves[3], s, p, d, g, dg, mask=mm)
        (y * gy.to(dev, dt)).sum().backward()
        outs.append([y] + [t.grad for t in leaves] + ([mm.grad] if mm is not None else []))
    for k, (a, r) in enumerate(zip(*outs)):
        assert _rel(a.cpu().double(), r) < 1e-4, (k, _rel(a.cpu().double(), r), a.shape)
