#!/usr/bin/env python
"""HIP flash attention vs PyTorch SDPA (bf16) on ViT shapes: forward and
forward+backward, hipGraph-timed (no launch overhead).

    python scripts/attn_microbench.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_time(fn, iters):
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from mdistiller_ddp_amd.ops import attention as A
    from mdistiller_ddp_amd.ops.backend import use_backend
    for name, B, H in (("vit_tiny b256", 256, 3), ("vit_small b128", 128, 6), ("vit_base b64", 64, 12)):
        N = 197
        qkv = torch.randn(B, N, 3 * H * 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
        go = torch.randn(B, N, H * 64, device="cuda").to(torch.bfloat16)
        flop_f = 4.0 * B * H * N * N * 64
        row = {"shape": name, "B": B, "H": H, "N": N}
        for tag, be in (("hip", "hip"), ("sdpa", "torch")):
            def fwd():
                with use_backend(be):
                    return A.attention(qkv, H)

            def fwdbwd():
                with use_backend(be):
                    o = A.attention(qkv, H)
                torch.autograd.grad(o, qkv, go)
            with torch.no_grad():
                tf = graph_time(fwd, a.iters)
            tb = graph_time(fwdbwd, a.iters)
            row[f"{tag}_fwd_us"] = round(tf, 2)
            row[f"{tag}_fwdbwd_us"] = round(tb, 2)
            row[f"{tag}_fwd_tflops"] = round(flop_f / tf / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
