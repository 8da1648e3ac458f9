#!/usr/bin/env python
"""Phase breakdown (in-kernel s_memrealtime stamps) of one conv dgrad launch,
per strided-dgrad parity class: prologue, first stage landed, main loop,
epilogue.  Also times the launch in a hipGraph.

    python scripts/dgrad_stamps.py --shape N,Cin,H,Cout,k,s [--runs 3]
"""
import argparse
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="64,128,16,256,3,2")
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--op", default="dgrad", choices=["dgrad", "fwd", "bnsum", "fold"],
                    help="bnsum: dgrad + the consumer-BN sums epilogue (ReLU + residual); fold: "
                         "bnsum with the stride-s 1x1 shortcut dgrad folded in (mda_conv_dgrad_bnsum2)")
    a = ap.parse_args()
    N, Cin, H, Cout, k, s = map(int, a.shape.split(","))
    p = k // 2
    from mdistiller_ddp_amd.ops import _ext, hip_train
    from mdistiller_ddp_amd.ops.hip_layers import conv_plan
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
    Ho = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wf, wt, Kp, KpT = hip_train.pack_weights(conv.weight, True)
    dx = torch.empty(N, Cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if a.op in ("bnsum", "fold"):
        bn_y = torch.randn_like(dx)
        bn_res = torch.randn_like(dx)
        stats = torch.rand(4, Cin, device="cuda") + 0.5
        region = torch.zeros(hip_train._region_bytes(Cin) // 4, dtype=torch.float32, device="cuda")
        sc = nn.Conv2d(Cin, Cout, 1, s, 0, bias=False).cuda()
        _, wt2, _, kp2 = hip_train.pack_weights(sc.weight, True)
        dy2 = torch.randn_like(dy)
    if a.op in ("dgrad", "bnsum", "fold"):
        tile, splits = conv_plan(N * H * H, Cin, KpT)
        part = torch.empty(splits * N * H * H * Cin, device="cuda") if splits > 1 else None
    else:
        tile, splits = conv_plan(N * Ho * Ho, Cout, Kp)
        part = torch.empty(splits * N * Ho * Ho * Cout, device="cuda") if splits > 1 else None
        x = dx.normal_()
        y = torch.empty_like(dy)

    def run():
        if a.op == "bnsum":
            _ext.call("mda_conv_dgrad_bnsum", dy, wt, dx, part, None, N, H, H, Cin, Ho, Ho, Cout, k, k,
                      s, p, KpT, tile, splits, bn_y, bn_res, stats, 1, region)
        elif a.op == "fold":
            _ext.call("mda_conv_dgrad_bnsum2", dy, wt, dx, N, H, H, Cin, Ho, Ho, Cout, k, k, s, p, KpT,
                      bn_y, bn_res, stats, 1, region, None, dy2, wt2, Cout, kp2)
        elif a.op == "dgrad":
            _ext.call("mda_conv_dgrad", dy, wt, dx, part, N, H, H, Cin, Ho, Ho, Cout, k, k, s, p, KpT,
                      tile, splits)
        else:
            _ext.call("mda_conv_fwd", x, wf, None, None, None, y, None, part, N, H, H, Cin, Ho, Ho,
                      Cout, k, k, s, p, Kp, 1, tile, splits)
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
    print(f"{a.op} shape {a.shape} tile {tile} splits {splits}: {e0.elapsed_time(e1) * 1000 / 20:.2f} us/launch (graph)")
    buf = torch.zeros(8192 * 8, dtype=torch.int64, device="cuda")
    gx = None
    for r in range(a.runs):
        buf.zero_()
        torch.cuda.synchronize()
        _ext.call("mda_conv_set_stamps", buf)
        run()
        _ext.call("mda_conv_set_stamps", None)
        torch.cuda.synchronize()
        st = buf.view(-1, 8).cpu()
        nb = int((st[:, 0] > 0).nonzero().max().item()) + 1 if (st[:, 0] > 0).any() else 0
        if nb == 0:
            print("no stamps")
            return
        st = st[:nb].double() * 10.0 / 1000.0
        live = st[:, 0] > 0
        t0 = st[live, 0].min()
        bm = tile // 1000
        if a.op != "fwd":
            mc = N * ((H + s - 1) // s) ** 2 if s > 1 else N * H * H
            gy = (Cin + tile % 1000 - 1) // (tile % 1000)
        else:
            mc = N * Ho * Ho
            gy = (Cout + tile % 1000 - 1) // (tile % 1000)
        gx = (mc + bm - 1) // bm
        per_z = gx * gy
        print(f"run {r}: blocks {int(live.sum())} of {nb}  span {(st[live, 4] - t0).max().item():.2f} us")
        q = lambda v: f"{v.median().item():6.2f} [{v.min().item():6.2f},{v.max().item():6.2f}]"
        nz = (nb + per_z - 1) // per_z
        for z in range(nz):
            sl = st[z * per_z:(z + 1) * per_z]
            sl = sl[sl[:, 0] > 0]
            if len(sl) == 0:
                continue
            rel = sl - t0
            print(f"  z={z} ({len(sl)} blocks): start {q(rel[:, 0])} issue {q(rel[:, 1] - rel[:, 0])} "
                  f"land0 {q(rel[:, 2] - rel[:, 1])} loop {q(rel[:, 3] - rel[:, 2])} "
                  f"epi {q(rel[:, 4] - rel[:, 3])} end {q(rel[:, 4])}")


if __name__ == "__main__":
    main()
