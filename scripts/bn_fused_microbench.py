"""Fused training-BN kernels on the student's shapes, graph-captured back to
back and event-timed:

  bwd    mda_bn_bwd_fused (one grid-barrier launch) vs the 2-launch
         partial-rows path (mda_bn_bwd_reduce2 + mda_bn_bwd_apply)
  apply  mda_bn_apply_fin (finalize in the prologue)
  copy   torch add of two tensors (read 2, write 1): the streaming floor

usage: python scripts/bn_fused_microbench.py
"""
import torch

from mdistiller_ddp_amd.ops import _ext, hip_train

dev = "cuda"
SHAPES = [(65536, 32), (65536, 64), (16384, 128), (4096, 256)]
REPS = 40


def timed(fn, pre=None):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        if pre:
            pre()
        for i in range(REPS):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        if pre:
            pre()
        for i in range(REPS):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / (5 * REPS)


def main():
    _ext.load(required=True)
    print(f"{'M':>6} {'C':>5} | {'bwd fused':>9} {'bwd 2-launch':>12} | {'apply_fin':>9} {'stats_acc':>9} | {'add floor':>9}  (us)")
    for M, C in SHAPES:
        y = torch.randn(M, C, device=dev).bfloat16()
        dout = torch.randn(M, C, device=dev).bfloat16()
        res = torch.randn(M, C, device=dev).bfloat16()
        dy = torch.empty_like(y)
        dres = torch.empty_like(y)
        out = torch.empty_like(y)
        stats = torch.stack([y.float().mean(0), y.float().var(0).add(1e-5).rsqrt(),
                             torch.rand(C, device=dev), torch.rand(C, device=dev)]).contiguous()
        g_, b_ = torch.rand(C, device=dev), torch.rand(C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        rb = hip_train._region_bytes(C)
        regions = torch.zeros(REPS * rb, dtype=torch.uint8, device=dev)
        err = torch.zeros(4, dtype=torch.int32, device=dev)
        part = torch.zeros(2 * 2048 * 512, device=dev)
        sums = torch.zeros(2, C, device=dev)
        zero = lambda: regions.zero_()  # noqa: E731

        def bwd_fused(i):
            _ext.call("mda_bn_bwd_fused", dout, None, None, y, res, stats, M, C, 1,
                      regions[i * rb:(i + 1) * rb], err, dy, dres, dg, db, None, None, None, None, None,
                      1, 0, 0, 0)

        def bwd_old(i):
            _ext.call("mda_bn_bwd_reduce2", dout, None, y, res, stats[2], stats[3], stats[0], stats[1],
                      M, C, 1, part, sums, dg, db)
            _ext.call("mda_bn_bwd_apply", dout, None, y, res, stats[2], stats[3], stats[0], stats[1],
                      sums, dy, dres, M, C, 1)

        st4 = torch.zeros(4, C, device=dev)

        def apply(i):
            _ext.call("mda_bn_apply_fin", y, regions[i * rb:(i + 1) * rb], M, C, g_, b_, None, None,
                      st4, 0.1, 1e-5, None, res, out, None, 1)

        def stats_acc(i):
            _ext.call("mda_bn_stats_acc", y, M, C, regions[i * rb:(i + 1) * rb])

        def add(i):
            torch.add(y, dout, out=out)

        t_zero = timed(lambda i: None, pre=zero)  # memset alone, amortised per rep
        t = [timed(bwd_fused, zero) - t_zero, timed(bwd_old), timed(apply, zero) - t_zero,
             timed(stats_acc, zero) - t_zero, timed(add)]
        torch.cuda.synchronize()
        assert int(err.max()) == 0, "grid barrier timed out"
        print(f"{M:6d} {C:5d} | {t[0]:9.2f} {t[1]:12.2f} | {t[2]:9.2f} {t[3]:9.2f} | {t[4]:9.2f}")


if __name__ == "__main__":
    main()
