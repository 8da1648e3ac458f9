"""Would one launch doing a layer's dgrad AND wgrad beat the two in sequence?

For each conv of the ResNet8x4 student at batch 64 (the flagship backward),
captures (a) dgrad then wgrad on one stream, (b) the two as single-chain graphs
on two streams replayed together (what a horizontally fused kernel can at best
achieve), and (c) each alone.  Prints us per replay of a 20-layer-deep repeat.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mdistiller_ddp_amd.ops import _ext, hip_train  # noqa: E402
from mdistiller_ddp_amd.ops.hip_layers import conv_plan  # noqa: E402

SHAPES = [  # N, Cin, H, Cout, k, s, p  (ResNet8x4 student)
    (64, 32, 32, 64, 3, 1, 1),
    (64, 64, 32, 64, 3, 1, 1),
    (64, 32, 32, 64, 1, 1, 0),
    (64, 64, 32, 128, 3, 2, 1),
    (64, 128, 16, 128, 3, 1, 1),
    (64, 64, 32, 128, 1, 2, 0),
    (64, 128, 16, 256, 3, 2, 1),
    (64, 256, 8, 256, 3, 1, 1),
    (64, 128, 16, 256, 1, 2, 0),
]
REP = 10


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / it


def main():
    _ext.load(required=True)
    dev = "cuda"
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    tot = {"seq": 0.0, "par": 0.0, "d": 0.0, "w": 0.0}
    for (N, Cin, H, Cout, k, s, p) in SHAPES:
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, Cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, Cout, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        _, wt, Kp, KpT = hip_train.pack_weights(w, True)
        dx = torch.empty_like(x)
        tile, splits = conv_plan(N * H * H, Cin, KpT)
        part = torch.empty(splits * N * H * H * Cin, dtype=torch.float32, device=dev) if splits > 1 else None
        M = N * Ho * Ho
        sp = hip_train._wgrad_splits(M, Cout, Cin, k, k, Kp, H, H, s, p)
        wpart = torch.empty(sp * Cout * Kp, dtype=torch.float32, device=dev)
        grad = torch.zeros(Cout, Cin, k, k, device=dev)

        def dg():
            _ext.call("mda_conv_dgrad", dy, wt, dx, part, N, H, H, Cin, Ho, Ho, Cout, k, k, s, p, KpT,
                      tile, splits)

        def wg():
            _ext.call("mda_conv_wgrad_nored", x, dy, wpart, grad, N, H, H, Cin, Ho, Ho, Cout, k, k, s,
                      p, Kp, sp, 1.0, 1, 0, 1, 1)

        graphs = {}
        for name, fns, st in (("seq", (dg, wg), s1), ("d", (dg,), s1), ("w", (wg,), s2)):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                for f in fns:
                    f()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(REP):
                    for f in fns:
                        f()
            graphs[name] = g
        res = {}
        res["seq"] = timeit(graphs["seq"].replay) / REP
        res["d"] = timeit(graphs["d"].replay) / REP
        res["w"] = timeit(graphs["w"].replay) / REP

        def par():
            s2.wait_stream(cur)
            with torch.cuda.stream(s2):
                graphs["w"].replay()
            graphs["d"].replay()
            cur.wait_stream(s2)
        res["par"] = timeit(par) / REP
        for kk in tot:
            tot[kk] += res[kk]
        print(f"{Cin:4d}->{Cout:4d} k{k} s{s} {H:3d}px: dgrad {res['d']:6.1f}  wgrad {res['w']:6.1f}  "
              f"seq {res['seq']:6.1f}  concurrent {res['par']:6.1f} us", flush=True)
    print(f"total: dgrad {tot['d']:.1f} wgrad {tot['w']:.1f} seq {tot['seq']:.1f} concurrent {tot['par']:.1f} us")


if __name__ == "__main__":
    main()
