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


if __name__ == "__main__":
    main()
