"""Per-kernel floor of a replayed hipGraph on this GPU: N dependent tiny
kernels (one 1-block add each) captured on one stream; replay time / N is the
cost a kernel boundary adds to a latency-bound chain.  Also the same chain with
a 512-block elementwise kernel (a small activation of the CIFAR student) and
two independent chains on a forked stream."""
import time

import torch


def timeit(fn, it=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


def main():
    dev = "cuda"
    s = torch.cuda.Stream()
    for numel, label in ((1, "1-block add"), (64 * 32 * 32 * 64, "4M-elt bf16 add (512+ blocks)")):
        x = torch.zeros(numel, device=dev, dtype=torch.bfloat16)
        for n in (50, 200):
            with torch.cuda.stream(s):
                for _ in range(n):
                    x.add_(1)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    x.add_(1)
            us = timeit(g.replay)
            print(f"{label:32s} n={n:4d}: replay {us:8.1f} us  -> {us / n:6.2f} us/kernel", flush=True)
    # two independent chains, one forked onto a side stream inside the graph
    x = torch.zeros(1, device=dev)
    y = torch.zeros(1, device=dev)
    side = torch.cuda.Stream()
    n = 100
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        side.wait_stream(s)
        with torch.cuda.stream(side):
            for _ in range(n):
                y.add_(1)
        for _ in range(n):
            x.add_(1)
        s.wait_stream(side)
    us = timeit(g.replay)
    print(f"two forked 1-block chains n={n}: replay {us:8.1f} us -> {us / n:6.2f} us/kernel-pair", flush=True)
    # the same two chains as two single-chain graphs replayed on two streams
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=s):
        for _ in range(n):
            x.add_(1)
    with torch.cuda.graph(gb, stream=side):
        for _ in range(n):
            y.add_(1)
    cur = torch.cuda.current_stream()
    ev = [torch.cuda.Event() for _ in range(2)]

    def two():
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            gb.replay()
        ga.replay()
        cur.wait_stream(side)
    us = timeit(two)
    print(f"two graphs on two streams n={n}: replay {us:8.1f} us -> {us / n:6.2f} us/kernel-pair", flush=True)
    for pr in (-1, 0):
        hi = torch.cuda.Stream(priority=pr)
        lo = torch.cuda.Stream(priority=0)
        print(f"stream priority range {torch.cuda.Stream.priority_range()}", flush=True)
        # a big 4M-element chain on the low stream, tiny chain on the high stream
        z = torch.zeros(64 * 32 * 32 * 64, device=dev, dtype=torch.bfloat16)
        gz, gx = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gz, stream=lo):
            for _ in range(n):
                z.add_(1)
        with torch.cuda.graph(gx, stream=hi):
            for _ in range(n):
                x.add_(1)
        def alone():
            hi.wait_stream(cur)
            with torch.cuda.stream(hi):
                gx.replay()
            cur.wait_stream(hi)
        def both():
            lo.wait_stream(cur)
            hi.wait_stream(cur)
            with torch.cuda.stream(lo):
                gz.replay()
            with torch.cuda.stream(hi):
                gx.replay()
            cur.wait_stream(hi)
            t_hi = None
            cur.wait_stream(lo)
        us_a = timeit(alone)
        # time of the tiny (high) chain while the big chain runs beside it
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            both()
        torch.cuda.synchronize()
        lo.wait_stream(cur); hi.wait_stream(cur)
        with torch.cuda.stream(lo):
            gz.replay()
        with torch.cuda.stream(hi):
            e0.record(hi)
            gx.replay()
            e1.record(hi)
        torch.cuda.synchronize()
        print(f"priority {pr}: tiny chain alone {us_a:7.1f} us, beside a 4M-elt chain {e0.elapsed_time(e1) * 1e3:7.1f} us;"
              f" both {timeit(both):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
