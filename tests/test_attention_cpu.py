"""CPU path of ops.attention (the PyTorch fallback the ViT uses off-GPU) vs an
explicit softmax(q k^T / sqrt(d)) v, and the fused-qkv layout contract."""
import torch

from mdistiller_ddp_amd.ops import attention as A


def test_attention_fallback_matches_explicit_softmax():
    torch.manual_seed(0)
    B, N, H, D = 2, 11, 3, 64
    qkv = torch.randn(B, N, 3 * H * D, dtype=torch.float64)
    out = A.attention(qkv, H)
    q, k, v = qkv.view(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    p = torch.softmax(q @ k.transpose(-1, -2) / D ** 0.5, -1)
    ref = (p @ v).transpose(1, 2).reshape(B, N, H * D)
    torch.testing.assert_close(out, ref)
    assert not A.native_ok(qkv, H)  # CPU tensors never take the HIP path
