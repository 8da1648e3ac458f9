"""Which part of the KDSVD loss breaks hipGraph capture: captures growing
prefixes of the computation in one process (the first crash names the stage)."""
import sys

import torch

from mdistiller_ddp_amd.ops import _ext
from mdistiller_ddp_amd.ops import feat_losses as FL

_ext.load(required=True)
torch.manual_seed(0)
fs = torch.randn(64, 32, 32, 32, device="cuda", requires_grad=True)
ft = torch.randn(64, 64, 32, 32, device="cuda")
fs2 = torch.randn(64, 64, 16, 16, device="cuda", requires_grad=True)
ft2 = torch.randn(64, 128, 16, 16, device="cuda")
x = fs.detach().reshape(64, 1024, 32)
fs3 = torch.randn(64, 128, 8, 8, device="cuda", requires_grad=True)
ft3 = torch.randn(64, 256, 8, 8, device="cuda")
x8 = ft3.reshape(64, 2048, 8)


def eig8():
    g = torch.bmm(x8.transpose(1, 2), x8).contiguous()
    lam = torch.empty(64, 8, device="cuda")
    v = torch.empty(64, 8, 8, device="cuda")
    _ext.call("mda_sym_eig", g, 64, 8, 8, lam, v)
    return v


def eig_only():
    g = torch.bmm(x.transpose(1, 2), x).contiguous()
    lam = torch.empty(64, 32, device="cuda")
    v = torch.empty(64, 32, 32, device="cuda")
    _ext.call("mda_sym_eig", g, 64, 32, 8, lam, v)
    return v


STAGES = [
    ("bmm8", lambda: torch.bmm(x8.transpose(1, 2), x8)),
    ("eig8", eig8),
    ("loss3_fwd_bwd", lambda: FL.kdsvd_loss([fs, fs2, fs3], [ft, ft2, ft3], 1).backward()),
    ("bmm", lambda: torch.bmm(x.transpose(1, 2), x)),
    ("eig", eig_only),
    ("svd_gram_fwd", lambda: FL._svd_gram(fs.detach(), 4)[2]),
    ("loss_fwd_nograd", lambda: FL.kdsvd_loss([fs.detach(), fs2.detach()], [ft, ft2], 1)),
    ("loss_fwd", lambda: FL.kdsvd_loss([fs, fs2], [ft, ft2], 1)),
    ("loss_fwd_bwd", lambda: FL.kdsvd_loss([fs, fs2], [ft, ft2], 1).backward()),
]
only = sys.argv[1:] or [n for n, _ in STAGES]
for name, fn in STAGES:
    if name not in only:
        continue
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    fs.grad = fs2.grad = fs3.grad = None
    print("capturing", name, flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        fn()
    g.replay()
    torch.cuda.synchronize()
    print("ok", name, flush=True)
