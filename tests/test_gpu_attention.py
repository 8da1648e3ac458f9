"""HIP flash attention (csrc/attention.hip) vs an fp32 PyTorch reference:
forward output and the fused d(qkv) gradient, ViT sequence lengths (197),
tile tails and tiny sequences; plus the ViT block end to end on the native path."""
import pytest
import torch

from mdistiller_ddp_amd.ops import attention as A
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B,N,H", [(2, 197, 3), (3, 64, 2), (1, 5, 1), (2, 130, 6), (1, 257, 4)])
def test_flash_attention_fwd_bwd(B, N, H):
    torch.manual_seed(0)
    qkv = (torch.randn(B, N, 3 * H * 64, device=DEV) * 1.5).to(torch.bfloat16)
    go = torch.randn(B, N, H * 64, device=DEV).to(torch.bfloat16)
    x = qkv.clone().requires_grad_(True)
    with use_backend("hip"):
        assert A.native_ok(x, H)
        out = A.attention(x, H)
    out.backward(go)
    xr = qkv.float().clone().requires_grad_(True)
    ref = A.attention_ref(xr, H)
    ref.backward(go.float())
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    err = (x.grad.float() - xr.grad).norm() / xr.grad.norm()
    assert err < 2e-2, float(err)
    # every block of d(qkv) is populated (q, k and v parts)
    g = x.grad.float().view(B, N, 3, H, 64)
    for part in range(3):
        assert g[:, :, part].abs().sum() > 0


def test_vit_block_native_matches_torch():
    from mdistiller_ddp_amd.models.imagenet.vit import Block
    torch.manual_seed(1)
    blk = Block(384, 6).to(DEV)
    x = torch.randn(2, 197, 384, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        with use_backend("hip"):
            y = blk(x)
        with use_backend("torch"):
            y_ref = blk(x)
    torch.testing.assert_close(y.float(), y_ref.float(), atol=5e-2, rtol=5e-2)
