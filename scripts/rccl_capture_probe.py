"""Probe: is an RCCL all-reduce capturable into a hipGraph with this torch/RCCL?
One rank (RCCL rejects two ranks on one device), so it checks the capture
mechanics, not cross-GPU traffic.  Run under ``timeout``."""
import os
import socket

import torch
import torch.distributed as dist


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), WORLD_SIZE="1",
                      RANK="0")
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    y = torch.arange(1 << 20, device=dev, dtype=torch.float32)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):
            z = y * 1.0
            w = dist.all_reduce(z, async_op=True)
            w.wait()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        z = y * 1.0
        w = dist.all_reduce(z, async_op=True)
        w.wait()
        z2 = z * 2.0
    for i in range(3):
        y.add_(1.0)
        g.replay()
    torch.cuda.synchronize()
    ok = torch.equal(z2, (y * 2.0))
    print(f"captured all_reduce (async + wait) replay ok={ok}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
