"""hipBLASLt reference: bf16 GEMMs with the teacher convs' implicit-GEMM shapes
(M = N*Ho*Wo, K = 9*Cin, N = Cout) -- the library-GEMM bar for conv kernels.
Run under rocprofv3 --kernel-trace for per-kernel times."""
import torch

SHAPES = [(65536, 576, 64), (16384, 1152, 128), (4096, 2304, 256), (65536, 288, 64)]
for M, K, N in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(30):
        c = a @ b
    torch.cuda.synchronize()
print("done")
