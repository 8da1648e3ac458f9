#!/usr/bin/env python
"""Phase breakdown (in-kernel s_memrealtime stamps) of the halo weight-gradient
kernel for one conv shape: prologue, first stage landed, main loop, partial
stores.  Also times the GEMM-only launch (no reduce) in a hipGraph.

    python scripts/wgrad_stamps.py --shape N,Cin,H,Cout [--runs 2]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,256,8,256")
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    N, Cin, H, Cout = map(int, a.shape.split(","))
    from mdistiller_ddp_amd.ops import _ext
    k, s, p = 3, 1, 1
    Kp = 9 * Cin
    M = N * H * H
    sp_ = ctypes.c_int64(0)
    _ext.call("mda_wgrad_plan", M, Cout, Cin, k, k, Kp, H, H, s, p, sp_)
    sp = sp_.value
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Cout, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    part = torch.empty(sp * Cout * Kp, device="cuda")
    grad = torch.zeros(Cout, Cin, k, k, device="cuda")

    def run():
        _ext.call("mda_conv_wgrad_nored", x, dy, part, grad, N, H, H, Cin, H, H, Cout, k, k, s, p, Kp,
                  sp, 1.0, 1, 0, 1, 1)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st_ = torch.cuda.Stream()
    with torch.cuda.stream(st_):
        with torch.cuda.graph(g, stream=st_):
            for _ in range(20):
                run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"wgrad shape {a.shape} splits {sp}: {e0.elapsed_time(e1) * 1000 / 20:.2f} us/launch (graph, no reduce)")
    buf = torch.zeros(8192 * 8, dtype=torch.int64, device="cuda")
    for r in range(a.runs):
        buf.zero_()
        torch.cuda.synchronize()
        _ext.call("mda_conv_set_stamps", buf)
        run()
        _ext.call("mda_conv_set_stamps", None)
        torch.cuda.synchronize()
        st = buf.view(-1, 8).cpu()
        live = st[:, 0] > 0
        if not live.any():
            print("no stamps")
            return
        st = st[live].double() * 10.0 / 1000.0
        t0 = st[:, 0].min()
        rel = st - t0
        q = lambda v: f"{v.median().item():6.2f} [{v.min().item():6.2f},{v.max().item():6.2f}]"
        print(f"run {r}: blocks {len(st)}  span {rel[:, 4].max().item():.2f} us  start {q(rel[:, 0])} "
              f"issue {q(rel[:, 1] - rel[:, 0])} land0 {q(rel[:, 2] - rel[:, 1])} loop {q(rel[:, 3] - rel[:, 2])} "
              f"store {q(rel[:, 4] - rel[:, 3])}")


if __name__ == "__main__":
    main()
