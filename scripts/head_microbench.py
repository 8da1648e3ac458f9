"""Time the fused pool+FC head kernels at the CIFAR flagship / ImageNet shapes (graph-replayed)."""
import torch

from mdistiller_ddp_amd.ops import _ext


def bench(fn, iters=200):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters // 20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


for (N, HW, C, J) in [(64, 64, 256, 100), (64, 49, 512, 1000), (64, 49, 1024, 1000)]:
    x = torch.randn(N, HW, C, device="cuda").to(torch.bfloat16)
    W = torch.randn(J, C, device="cuda") * 0.05
    b = torch.randn(J, device="cuda")
    pooled = torch.empty(N, C, device="cuda", dtype=torch.bfloat16)
    logits = torch.empty(N, J, device="cuda", dtype=torch.bfloat16)
    dl = torch.randn(N, J, device="cuda").to(torch.bfloat16)
    dW = torch.zeros(J, C, device="cuda")
    db = torch.zeros(J, device="cuda")
    dx = torch.empty_like(x)
    tf = bench(lambda: _ext.call("mda_pool_fc_fwd", 1, x, W, b, pooled, logits, N, HW, C, J))
    tb = bench(lambda: _ext.call("mda_pool_fc_bwd", 1, dl, None, pooled, W, dW, db, dx, N, HW, C, J, 0))
    ref = (x.float().mean(1).to(torch.bfloat16).float() @ W.t() + b)
    err = ((logits.float() - ref).abs().max() / ref.abs().max()).item()
    print(f"N={N} HW={HW} C={C} J={J}: fwd {tf:.2f} us  bwd {tb:.2f} us  fwd rel err {err:.2e}", flush=True)
