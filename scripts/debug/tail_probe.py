"""Where does the ShuffleV1 tail backward put a unit gradient?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.ops import _ext  # noqa: E402

N, C3, Cx, H = 1, 8, 8, 4
W, Ho, Wo = H, 2, 2
cl = torch.channels_last
pre = torch.ones(N, C3 + Cx, Ho, Wo, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
for oh in range(Ho):
    for ow in range(Wo):
        dout = torch.zeros_like(pre)
        dout[0, C3, oh, ow] = 9.0
        dy3 = torch.empty(N, C3, Ho, Wo, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        dx = torch.empty(N, Cx, H, W, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        _ext.call("mda_shuffle_tail_bwd", dout, None, pre, dy3, dx, N, H, W, Ho, Wo, C3, Cx)
        torch.cuda.synchronize()
        nz = (dx[0, 0].float() != 0).nonzero().tolist()
        print(f"unit grad at out ({oh},{ow}) -> dx nonzero at {nz} (expect rows/cols {2*oh-1}..{2*oh+1})", flush=True)
