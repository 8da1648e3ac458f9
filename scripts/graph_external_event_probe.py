"""Can a stream outside a replayed hipGraph wait on an event recorded in the
MIDDLE of that graph?  (``hipEventRecordExternal`` through csrc/events.hip:
PyTorch's ROCm build refuses ``torch.cuda.Event(external=True)``.)

This is what an all-reduce overlapped with a captured backward needs: the
graph records "bucket k complete" and the comm stream, enqueued by the host
right after the replay, waits on it.  Checks ordering (the snapshot taken on
the side stream equals the value at the record point of THIS replay, never an
older one) and timing (the side work finishes well before the graph does).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdistiller_ddp_amd.runtime.streams import HipEvent  # noqa: E402


def main():
    dev = "cuda"
    s, side = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    x = torch.zeros(1, device=dev)
    y = torch.zeros(1, device=dev)
    z = torch.zeros(1, device=dev)
    n = 200
    ev = HipEvent()
    with torch.cuda.stream(s):
        x.add_(1)
    torch.cuda.synchronize()
    x.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            x.add_(1)
        ev.record(external=True)
        for _ in range(n):
            y.add_(1)
    torch.cuda.synchronize()
    x.zero_()
    y.zero_()
    torch.cuda.synchronize()
    ok = True
    t_side, t_all = [], []
    for k in range(1, 21):
        t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        t0.record(s)
        with torch.cuda.stream(s):
            g.replay()
        t2.record(s)
        ev.wait(side)
        with torch.cuda.stream(side):
            z.copy_(x)
            t1.record(side)
        torch.cuda.synchronize()
        zv, xv = float(z), float(x)
        if zv != n * k:
            ok = False
            print(f"replay {k}: side snapshot {zv}, expected {n * k} (x now {xv})", flush=True)
        t_side.append(t0.elapsed_time(t1) * 1e3)
        t_all.append(t0.elapsed_time(t2) * 1e3)
    print(f"external event mid-graph: ordering {'OK' if ok else 'BROKEN'}; side work done at "
          f"{sorted(t_side)[10]:.1f} us of a {sorted(t_all)[10]:.1f} us replay", flush=True)


if __name__ == "__main__":
    for mode in (2, 1):
        HipEvent.MODE = mode
        try:
            print(f"-- record/wait mode {mode}", flush=True)
            main()
        except RuntimeError as e:
            print(f"mode {mode}: {e}", flush=True)
    HipEvent.MODE = 2


def two_graph_events():
    """Graph A records an external event every 20 kernels; graph B, replayed
    concurrently on another stream, waits on each and snapshots x.  The
    pattern of a backward whose weight-gradient GEMMs run as a second graph."""
    dev = "cuda"
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(1, device=dev)
    snaps = torch.zeros(10, device=dev)
    w = torch.zeros(1, device=dev)
    evs = [HipEvent() for _ in range(10)]
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(sa):
        x.add_(1)
    torch.cuda.synchronize()
    with torch.cuda.graph(ga, stream=sa):
        for e in evs:
            for _ in range(20):
                x.add_(1)
            e.record(external=True)
    with torch.cuda.graph(gb, stream=sb):
        for i, e in enumerate(evs):
            e.wait(external=True)
            snaps[i].copy_(x[0])
            for _ in range(5):
                w.add_(1)
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream()
    bad = 0
    times = []
    for k in range(1, 21):
        x.zero_()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(cur)
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            ga.replay()
        with torch.cuda.stream(sb):
            gb.replay()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        t1.record(cur)
        torch.cuda.synchronize()
        want = torch.arange(1, 11, device=dev, dtype=torch.float32) * 20
        if not torch.equal(snaps, want):
            bad += 1
            if bad <= 3:
                print(f"replay {k}: snapshots {snaps.tolist()}", flush=True)
        times.append(t0.elapsed_time(t1) * 1e3)
    # reference: A alone
    ta0, ta1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ta0.record(cur)
    sa.wait_stream(cur)
    with torch.cuda.stream(sa):
        ga.replay()
    cur.wait_stream(sa)
    ta1.record(cur)
    torch.cuda.synchronize()
    print(f"two graphs with external events: ordering {'OK' if bad == 0 else f'BROKEN in {bad}/20'}; "
          f"both {sorted(times)[10]:.1f} us, graph A alone {ta0.elapsed_time(ta1) * 1e3:.1f} us "
          f"(200 + 10 events; B: 10 waits + 60 kernels)", flush=True)


if __name__ == "__main__":
    for mode in (2, 1):
        HipEvent.MODE = mode
        try:
            print(f"-- two graphs, mode {mode}", flush=True)
            two_graph_events()
        except RuntimeError as e:
            print(f"mode {mode}: {e}", flush=True)
