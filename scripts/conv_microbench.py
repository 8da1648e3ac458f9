#!/usr/bin/env python
"""Per-shape timing of the MFMA implicit-GEMM conv kernels vs MIOpen.

For every conv shape of the north-star pair (resnet32x4 teacher, resnet8x4
student) at batch 64: forward (inference epilogue), dgrad, wgrad; reports
us/call and TFLOP/s, and MIOpen's bf16 channels-last time for the same op.

    python scripts/conv_microbench.py [--iters 50] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # N, Cin, H, Cout, k, s, p
    (64, 3, 32, 32, 3, 1, 1),
    (64, 32, 32, 64, 3, 1, 1),
    (64, 64, 32, 64, 3, 1, 1),
    (64, 64, 32, 128, 3, 2, 1),
    (64, 128, 16, 128, 3, 1, 1),
    (64, 128, 16, 256, 3, 2, 1),
    (64, 256, 8, 256, 3, 1, 1),
    (64, 64, 32, 128, 1, 2, 0),
    (64, 128, 16, 256, 1, 2, 0),
    (64, 32, 32, 64, 1, 1, 0),
]
IMAGENET = [  # ResNet-50 teacher at batch 64, ResNet-18 student at batch 32
    (64, 64, 56, 64, 1, 1, 0),
    (64, 64, 56, 256, 1, 1, 0),
    (64, 256, 56, 64, 1, 1, 0),
    (64, 64, 56, 64, 3, 1, 1),
    (64, 256, 56, 512, 1, 2, 0),
    (64, 128, 28, 512, 1, 1, 0),
    (64, 512, 28, 128, 1, 1, 0),
    (64, 128, 28, 128, 3, 1, 1),
    (64, 1024, 14, 256, 1, 1, 0),
    (64, 256, 14, 1024, 1, 1, 0),
    (64, 512, 7, 2048, 1, 1, 0),
    (64, 2048, 7, 512, 1, 1, 0),
    (32, 64, 56, 64, 3, 1, 1),
    (32, 128, 28, 128, 3, 1, 1),
    (32, 256, 14, 256, 3, 1, 1),
    (32, 512, 7, 512, 3, 1, 1),
]
MV1 = [  # MobileNetV1 student pointwise convs at batch 64
    (64, 32, 112, 64, 1, 1, 0),
    (64, 64, 56, 128, 1, 1, 0),
    (64, 128, 56, 128, 1, 1, 0),
    (64, 128, 28, 256, 1, 1, 0),
    (64, 256, 28, 256, 1, 1, 0),
    (64, 256, 14, 512, 1, 1, 0),
    (64, 512, 14, 512, 1, 1, 0),
    (64, 512, 7, 1024, 1, 1, 0),
    (64, 1024, 7, 1024, 1, 1, 0),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def timeit_eager(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def timeit_graph(fn, iters):
    """GPU time per call with the Python/launch overhead removed: `iters`
    calls captured in one hipGraph, replayed."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--json", default=None)
    ap.add_argument("--shape", type=int, default=-1, help="index into SHAPES (-1 = all)")
    ap.add_argument("--ops", default="fwd,mio,wgrad,dgrad")
    ap.add_argument("--set", default="cifar", choices=["cifar", "imagenet", "mv1"])
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays (no CPU overhead)")
    args = ap.parse_args()
    global timeit
    if args.graph:
        timeit = timeit_graph
    ops = set(args.ops.split(","))
    from mdistiller_ddp_amd.ops import hip_layers, hip_train
    torch.backends.cudnn.benchmark = True
    rows = []
    table = {"cifar": SHAPES, "imagenet": IMAGENET, "mv1": MV1}[args.set]
    shapes = table if args.shape < 0 else [table[args.shape]]
    nan = float("nan")
    for (N, Cin, H, Cout, k, s, p) in shapes:
        conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
        bn = nn.BatchNorm2d(Cout).cuda().eval()
        x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        Ho = (H + 2 * p - k) // s + 1
        flop = 2.0 * N * Ho * Ho * Cout * Cin * k * k
        with torch.no_grad():
            t_fwd = timeit(lambda: hip_layers.conv_bn_act(x, conv, bn, "relu", None, False), args.iters) if "fwd" in ops else nan
            wb = conv.weight.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            t_mio = nan
            dy = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            t_wg = timeit(lambda: hip_train.conv_wgrad(x, dy, tuple(conv.weight.shape), s, p), args.iters) if "wgrad" in ops else nan
            t_dg = nan
            if Cin % 8 == 0 and "dgrad" in ops:
                t_dg = timeit(lambda: hip_train.conv_dgrad(dy, conv.weight, tuple(x.shape), s, p), args.iters)
        # MIOpen (bf16 channels-last) forward / dgrad / wgrad, timed eagerly
        # (its solvers are not capturable): event time per call over `iters`
        t_mio_dg = t_mio_wg = nan
        if "mio" in ops:
            wb = conv.weight.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            t_mio = timeit_eager(lambda: F.conv2d(x, wb, stride=s, padding=p), args.iters)
            t_mio_dg = timeit_eager(lambda: torch.ops.aten.convolution_backward(
                dy, x, wb, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (True, False, False)),
                args.iters)
            t_mio_wg = timeit_eager(lambda: torch.ops.aten.convolution_backward(
                dy, x, wb, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (False, True, False)),
                args.iters)
        row = dict(shape=[N, Cin, H, Cout, k, s, p], gflop=flop / 1e9, fwd_us=t_fwd,
                   fwd_tflops=flop / t_fwd / 1e6, miopen_fwd_us=t_mio, dgrad_us=t_dg,
                   wgrad_us=t_wg, wgrad_tflops=flop / t_wg / 1e6, dgrad_tflops=flop / t_dg / 1e6,
                   miopen_tflops=flop / t_mio / 1e6, miopen_dgrad_us=t_mio_dg,
                   miopen_wgrad_us=t_mio_wg)
        rows.append(row)
        print(json.dumps({k_: (round(v, 2) if isinstance(v, float) else v) for k_, v in row.items()}),
              flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
