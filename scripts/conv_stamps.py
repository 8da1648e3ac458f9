#!/usr/bin/env python
"""Phase breakdown of the instrumented conv kernel (halo2) from in-kernel
s_memrealtime stamps (100 MHz): launch skew, prologue (DMA issue), wait for
the patch + first weight tap, the 9-tap MFMA loop, epilogue.

    python scripts/conv_stamps.py [--shape N,Cin,H,Cout] [--dgrad]
"""
import argparse
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,64,32,64")
    ap.add_argument("--runs", type=int, default=5)
    a = ap.parse_args()
    N, Cin, H, Cout = map(int, a.shape.split(","))
    from mdistiller_ddp_amd.ops import _ext, hip_layers
    conv = nn.Conv2d(Cin, Cout, 3, 1, 1, bias=False).cuda().eval()
    bn = nn.BatchNorm2d(Cout).cuda().eval()
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        for _ in range(5):
            hip_layers.conv_bn_act(x, conv, bn, "relu", None, False)
        torch.cuda.synchronize()
        buf = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
        for r in range(a.runs):
            buf.zero_()
            torch.cuda.synchronize()
            _ext.call("mda_conv_set_stamps", buf)
            hip_layers.conv_bn_act(x, conv, bn, "relu", None, False)
            _ext.call("mda_conv_set_stamps", None)
            torch.cuda.synchronize()
            st = buf.view(-1, 8).cpu()
            st = st[st[:, 0] > 0].double() * 10.0 / 1000.0  # ticks of 10 ns -> us
            if len(st) == 0:
                print("no stamps (kernel not instrumented for this shape)")
                return
            t0 = st[:, 0].min()
            rel = st[:, :5] - t0
            q = lambda v: f"{v.median().item():6.2f} [{v.min().item():6.2f},{v.max().item():6.2f}]"
            print(f"run {r}: blocks {len(st)}  span {rel[:, 4].max().item():.2f} us")
            print("   start      ", q(rel[:, 0]))
            full = st - t0
            if (st[:, 5] > 0).all():  # multi-chunk halo kernel: prologue detail
                print("   epi prefetch", q(full[:, 5] - full[:, 0]))
                print("   addresses   ", q(full[:, 6] - full[:, 5]))
                print("   DMA issue   ", q(full[:, 1] - full[:, 6]))
            print("   issue done ", q(rel[:, 1] - rel[:, 0]))
            print("   tap0 landed", q(rel[:, 2] - rel[:, 1]))
            print("   9-tap loop ", q(rel[:, 3] - rel[:, 2]))
            print("   epilogue   ", q(rel[:, 4] - rel[:, 3]))
            print("   end        ", q(rel[:, 4]))


if __name__ == "__main__":
    main()
