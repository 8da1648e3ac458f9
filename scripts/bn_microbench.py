"""BN reduction kernels on the student's shapes: in-kernel two-level hand-off
(mda_bn_stats / mda_bn_bwd_reduce) vs partials + channel-parallel finalize
(mda_bn_stats2 / mda_bn_bwd_reduce2).  Graph-captured back-to-back calls,
event-timed; also checks the two variants agree."""
import torch

from mdistiller_ddp_amd.ops import _ext

dev = "cuda"
SHAPES = [(65536, 32), (65536, 64), (16384, 128), (4096, 256), (16384, 64), (4096, 128)]
REPS = 50


def timed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (5 * REPS)


import sys
VPT = int(sys.argv[1]) if len(sys.argv) > 1 else 8
MAXB = int(sys.argv[2]) if len(sys.argv) > 2 else 256
_ext.call("mda_bn_tune", VPT, MAXB)
print(f"vpt={VPT} max_blocks={MAXB}")
for M, C in SHAPES:
    y = torch.randn(M, C, device=dev).bfloat16()
    dout = torch.randn(M, C, device=dev).bfloat16()
    part = torch.zeros(2 * C * 4200, device=dev)
    cnt = torch.zeros(64, dtype=torch.int32, device=dev)
    g_, b_ = torch.rand(C, device=dev), torch.rand(C, device=dev)
    outs = [torch.zeros(4, C, device=dev) for _ in range(2)]
    sums = [torch.zeros(2, C, device=dev) for _ in range(2)]

    def st1():
        o = outs[0]
        _ext.call("mda_bn_stats", y, M, C, part, cnt, g_, b_, None, None, o[0], o[1], o[2], o[3],
                  0.1, 1e-5, None)

    def st2():
        o = outs[1]
        _ext.call("mda_bn_stats2", y, M, C, part, g_, b_, None, None, o[0], o[1], o[2], o[3],
                  0.1, 1e-5, None)

    def br1():
        o = outs[0]
        _ext.call("mda_bn_bwd_reduce", dout, None, y, None, o[2], o[3], o[0], o[1], M, C, 1, part,
                  cnt, sums[0], None, None)

    def br2():
        o = outs[0]
        _ext.call("mda_bn_bwd_reduce2", dout, None, y, None, o[2], o[3], o[0], o[1], M, C, 1, part,
                  sums[1], None, None)

    t = [timed(f) for f in (st1, st2, br1, br2)] if MAXB <= 256 else [0.0, timed(st2), 0.0, timed(br2)]
    torch.cuda.synchronize()
    d_st = (outs[0] - outs[1]).abs().max().item()
    d_br = ((sums[0] - sums[1]).abs().max() / sums[0].abs().max().clamp_min(1e-6)).item()
    print(f"M={M:6d} C={C:4d}  stats {t[0]:6.2f} -> {t[1]:6.2f} us   bwd_reduce {t[2]:6.2f} -> {t[3]:6.2f} us"
          f"   diff stats {d_st:.2e} bwd {d_br:.2e}")
