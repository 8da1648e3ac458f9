"""Localise VirtualBN differences: one downsampling BasicBlock, virtual
residual on / off / fp32 reference, every output and gradient."""
import copy
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.ops import hip_train  # noqa: E402
from mdistiller_ddp_amd.ops.backend import use_backend  # noqa: E402
from mdistiller_ddp_amd.models.cifar.resnet import BasicBlock  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def run(m, x, g, backend, preact):
    xx = x.clone().requires_grad_(True)
    with use_backend(backend), torch.autocast("cuda", dtype=torch.bfloat16, enabled=backend == "hip"):
        out, pre = m(xx if backend == "hip" else xx.float())
    loss = (out.float() * g).sum()
    loss.backward()
    torch.cuda.synchronize()
    return out, xx.grad


def main():
    for preact in (False, True):
        for (cin, cout, H) in ((64, 128, 32), (128, 256, 16)):
            torch.manual_seed(5)
            ds = nn.Sequential(nn.Conv2d(cin, cout, 1, 2, bias=False), nn.BatchNorm2d(cout))
            blk = BasicBlock(cin, cout, 2, ds, is_last=True).cuda().to(memory_format=torch.channels_last)
            blk._need_preact = preact
            off, ref = copy.deepcopy(blk), copy.deepcopy(blk)
            x = torch.randn(64, cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            g = torch.randn(64, cout, H // 2, H // 2, device="cuda")
            o1, d1 = run(blk, x, g, "hip", preact)
            hip_train.set_virtual_residual(False)
            o2, d2 = run(off, x, g, "hip", preact)
            hip_train.set_virtual_residual(True)
            o3, d3 = run(ref, x, g, "torch", preact)
            print(f"preact={preact} {cin}->{cout}: out v/off {rel(o1, o2):.4f} v/ref {rel(o1, o3):.4f} "
                  f"off/ref {rel(o2, o3):.4f} | dx v/off {rel(d1, d2):.4f} v/ref {rel(d1, d3):.4f} "
                  f"off/ref {rel(d2, d3):.4f}", flush=True)
            for (n, p), (_, q), (_, r) in zip(blk.named_parameters(), off.named_parameters(), ref.named_parameters()):
                print(f"    {n:22s} v/off {rel(p.grad, q.grad):.4f} v/ref {rel(p.grad, r.grad):.4f} "
                      f"off/ref {rel(q.grad, r.grad):.4f}", flush=True)
            for (n, b), (_, c), (_, r) in zip(blk.named_buffers(), off.named_buffers(), ref.named_buffers()):
                if b.dtype != torch.int64:
                    print(f"    {n:22s} v/off {rel(b, c):.4f} v/ref {rel(b, r):.4f}", flush=True)


if __name__ == "__main__":
    main()
