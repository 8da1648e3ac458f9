"""HIP CRD memory kernels and the CIFAR augmentation kernel vs PyTorch."""
import pytest
import torch

from mdistiller_ddp_amd.ops import crd as CO
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [64, 128])
def test_crd_scores_and_grad(D):
    torch.manual_seed(0)
    N, B, K1, T = 5000, 16, 4097, 0.07
    mem = torch.nn.functional.normalize(torch.randn(N, D, device="cuda"), dim=1)
    idx = torch.randint(0, N, (B, K1), device="cuda")
    v = torch.nn.functional.normalize(torch.randn(B, D, device="cuda"), dim=1)
    g = torch.randn(B, K1, device="cuda")
    v1 = v.clone().requires_grad_(True)
    with use_backend("hip"):
        e = CO.scores(mem, idx, v1, T)
    (e * g).sum().backward()
    v2 = v.clone().requires_grad_(True)
    e2 = CO.scores_ref(mem, idx, v2, T)
    (e2 * g).sum().backward()
    torch.testing.assert_close(e, e2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(v1.grad, v2.grad, rtol=1e-3, atol=1e-3)


def test_crd_update():
    torch.manual_seed(1)
    N, D, B = 1000, 128, 64
    mem = torch.randn(N, D, device="cuda")
    mem2 = mem.clone()
    y = torch.randperm(N, device="cuda")[:B]
    v = torch.randn(B, D, device="cuda")
    with use_backend("hip"):
        CO.update(mem, y, v, 0.5)
    CO.update_ref(mem2, y, v, 0.5)
    torch.testing.assert_close(mem, mem2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cifar_aug_kernel(dtype):
    from mdistiller_ddp_amd.data.cifar100 import DeviceImageLoader, augment_ref
    import numpy as np
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (100, 32, 32, 3), dtype=np.uint8)
    y = rng.integers(0, 100, 100)
    ld = DeviceImageLoader(x, y, 16, "cuda", train=True, out_dtype=dtype)
    idx = torch.arange(16, device="cuda") * 3
    torch.manual_seed(0)
    gen_state = ld.gen.get_state()
    with use_backend("hip"):
        out = ld._make(idx)
    ld.gen.set_state(gen_state)
    offs = torch.randint(0, 9, (16, 2), generator=ld.gen, device="cuda", dtype=torch.int32)
    flip = torch.randint(0, 2, (16,), generator=ld.gen, device="cuda", dtype=torch.uint8)
    ref = augment_ref(ld.x, idx, offs, flip)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    assert out.is_contiguous(memory_format=torch.channels_last)
