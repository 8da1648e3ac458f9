"""GradReducer's calibrated early bucket launches (parallel/grad_reducer.py)
on 2 gloo ranks: a parameter that receives TWO autograd contributions per
step (an autograd one and a native direct write) is reduced only after both landed, matching the
rank-mean of the local gradients; a later step that gives it a THIRD
contribution after its bucket was launched raises instead of silently
reducing stale values."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), MDA_BACKEND="torch")
    torch.set_num_threads(1)
    import torch.distributed as dist
    from mdistiller_ddp_amd.engine.optim import FlatParams
    from mdistiller_ddp_amd.parallel import dist as D
    from mdistiller_ddp_amd.parallel.grad_reducer import GradReducer
    D.init_distributed("gloo", 60.0, device="cpu")
    torch.manual_seed(0)
    shared = torch.nn.Linear(16, 16, bias=False)
    head = torch.nn.Linear(16, 4)
    params = list(shared.parameters()) + list(head.parameters())
    flat = FlatParams(params, 1)
    red = GradReducer(flat, bucket_mb=64 * 4 / (1 << 20), overlap=True)  # [head] [shared weight]
    out = {"buckets": len(red.buckets)}

    def grads(x):
        # autograd gradient + a second, "native" direct write of the shared
        # weight's gradient (as the HIP backward kernels do via notify_grad)
        loss = head(torch.tanh(shared(x))).square().mean()
        g = torch.autograd.grad(loss, params)
        return [g[0] + 0.5 * shared.weight.detach()] + list(g[1:])

    def step(extra_writes, seed):
        torch.manual_seed(seed + rank)
        x = torch.randn(8, 16)
        flat.zero_grad()
        red.arm()
        head(torch.tanh(shared(x))).square().mean().backward()  # autograd contribution
        for _ in range(extra_writes):
            with torch.no_grad():
                shared.weight.grad.add_(0.5 * shared.weight)
            red.ready_param(shared.weight)                        # direct-write contribution
        red.finish()
        return [t.clone() for t in grads(x)]

    step(1, 0)  # calibration: 2 contributions for the shared weight
    local = torch.cat([t.reshape(-1) for t in step(1, 1)])
    red_g = torch.cat([p.grad.reshape(-1) for p in params])
    allg = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    out["mean_ok"] = bool(torch.allclose(red_g, torch.stack(allg).sum(0), atol=1e-5))
    out["early"] = red.early_launches
    try:
        step(2, 2)
        out["raised"] = False
    except RuntimeError as e:
        out["raised"] = "contribution" in str(e)
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    D.destroy()


def test_reused_parameter_reduced_after_all_contributions_and_overflow_raises():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, _free_port(), td), nprocs=world, join=True)
        res = [torch.load(os.path.join(td, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in res:
        assert r["buckets"] >= 2
        assert r["mean_ok"], r
        assert r["early"] >= 1, r
        assert r["raised"], r


def test_auto_bucket_size_rule():
    """DIST.BUCKET_MB = 0: a quarter of the gradient, clamped to [0.5, 8] MB --
    four buckets for the flagship ResNet8x4 student, 8 MB ones for ResNet-18."""
    from mdistiller_ddp_amd.parallel.grad_reducer import auto_bucket_mb
    from mdistiller_ddp_amd.models.cifar import resnet8x4
    from mdistiller_ddp_amd.models.imagenet.resnet import resnet18
    n8 = sum(p.numel() for p in resnet8x4(num_classes=100).parameters())
    assert abs(auto_bucket_mb(n8) - n8 * 4 / (1 << 20) / 4) < 1e-9
    assert auto_bucket_mb(sum(p.numel() for p in resnet18().parameters())) == 8.0
    assert auto_bucket_mb(1000) == 0.5
