"""Is this ROCm build's channels_last avg_pool2d backward right?  The GPU
gradient of avg_pool2d(3, 2, 1) for NCHW and channels_last inputs vs the CPU
(fp32).  ShuffleNetV1's stride-2 shortcut is exactly this op."""
import torch
import torch.nn.functional as F


def grad(x, g):
    x = x.detach().requires_grad_(True)
    (F.avg_pool2d(x, 3, stride=2, padding=1) * g).sum().backward()
    return x.grad.float().cpu()


for dt in (torch.float32, torch.bfloat16):
    for (N, C, H) in ((2, 24, 32), (1, 8, 8)):
        torch.manual_seed(0)
        x = torch.randn(N, C, H, H)
        g = torch.randn(N, C, (H + 1) // 2, (H + 1) // 2)
        ref = grad(x, g)
        xg = x.cuda().to(dt)
        gg = g.cuda().to(dt)
        a = grad(xg.contiguous(), gg)
        b = grad(xg.contiguous(memory_format=torch.channels_last), gg.contiguous(memory_format=torch.channels_last))
        rel = lambda u: ((u - ref).norm() / ref.norm()).item()  # noqa: E731
        print(f"{dt} N={N} C={C} H={H}: NCHW rel {rel(a):.4f}  channels_last rel {rel(b):.4f}", flush=True)
        if rel(b) > 0.05:
            print("   row0 ref ", ref[0, 0, 0, :6].tolist(), "\n   row0 gpuCL", b[0, 0, 0, :6].tolist(), flush=True)
