"""Does a hipGraph with a fork/join (captured from two streams) execute its two
branches concurrently on this ROCm?  Compares replay time of:
  serial  - both chains captured on one stream
  fork    - chain A on the capture stream, chain B on a forked side stream
  twograph- each chain captured in its own graph, replayed on two streams
Chains are N small GEMMs that each occupy a few CUs, so true concurrency
shows up as ~2x."""
import time

import torch

N, S = 40, 256
dev = "cuda"
a = [torch.randn(S, S, device=dev, dtype=torch.bfloat16) for _ in range(2)]
w = torch.randn(S, S, device=dev, dtype=torch.bfloat16)


def chain(x):
    for _ in range(N):
        x = torch.tanh(x @ w)
    return x


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


main = torch.cuda.Stream()
side = torch.cuda.Stream()
with torch.cuda.stream(main):
    chain(a[0]); chain(a[1])
torch.cuda.synchronize()

g_serial = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_serial, stream=main):
    oa = chain(a[0]); ob = chain(a[1])

g_fork = torch.cuda.CUDAGraph()
with torch.cuda.graph(g_fork, stream=main):
    side.wait_stream(main)
    with torch.cuda.stream(side):
        ob2 = chain(a[1])
    oa2 = chain(a[0])
    main.wait_stream(side)

gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.graph(gA, stream=main):
    oa3 = chain(a[0])
with torch.cuda.graph(gB, stream=side):
    ob3 = chain(a[1])


def two():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        gB.replay()
    gA.replay()
    cur.wait_stream(side)


def one_chain():
    gA.replay()


print(f"one chain   {timeit(one_chain):8.1f} us")
print(f"serial      {timeit(g_serial.replay):8.1f} us")
print(f"fork graph  {timeit(g_fork.replay):8.1f} us")
print(f"two graphs  {timeit(two):8.1f} us")
