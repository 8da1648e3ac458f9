"""Probe: can two RCCL ranks share one GPU, and can an RCCL all-reduce be
captured into a hipGraph?  (Decides whether the single-GPU box can test the
``DIST.GRAPH_COMM=capture`` path.)  Run under ``timeout``.

Usage: python scripts/rccl_probe.py [world]
"""
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    t0 = time.time()
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    ok_eager = float(x[0]) == world * (world + 1) / 2
    print(f"[rank {rank}] eager all_reduce ok={ok_eager} ({time.time() - t0:.1f}s)", flush=True)
    # capture
    y = torch.full((1 << 20,), float(rank + 1), device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            z = y * 1.0
            dist.all_reduce(z)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, stream=s):
            z = y * 1.0
            dist.all_reduce(z)
            z2 = z * 2.0
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        ok_cap = float(z2[0]) == 2 * world * (world + 1) / 2
        print(f"[rank {rank}] captured all_reduce ok={ok_cap}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"[rank {rank}] capture failed: {type(e).__name__}: {e}", flush=True)
    dist.barrier(device_ids=[0])
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mp.start_processes(worker, args=(world, _port()), nprocs=world, join=True, start_method="spawn")
    print("probe done", flush=True)
