"""Fused multi-head self-attention for the ViT students (csrc/attention.hip).

``attention(qkv, num_heads)`` takes the fused projection output
``[B, N, 3 * H * 64]`` (bf16, as ``nn.Linear(dim, 3 * dim)`` produces it) and
returns ``softmax(q k^T / 8) v`` as ``[B, N, H * 64]``, ready for the output
projection.  On the HIP path the forward is one MFMA flash-attention launch
(no N x N matrix in memory); the backward recomputes the probabilities from
the saved log-sum-exp and writes ``d qkv`` in the same fused layout (three
launches).  Elsewhere (CPU, fp32, other head sizes) it is PyTorch SDPA.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .backend import hip_enabled_for

HEAD_DIM = 64


def native_ok(qkv: torch.Tensor, num_heads: int) -> bool:
    return (hip_enabled_for(qkv) and qkv.dtype == torch.bfloat16 and qkv.dim() == 3
            and qkv.shape[-1] == 3 * num_heads * HEAD_DIM)


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, num_heads, scale):
        from . import _ext
        qkv = qkv.contiguous()
        B, N, _ = qkv.shape
        H = num_heads
        o = torch.empty(B, N, H * HEAD_DIM, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * H * N, dtype=torch.float32, device=qkv.device)
        _ext.call("mda_attn_fwd", qkv, o, lse, B, N, H, float(scale))
        ctx.save_for_backward(qkv, o, lse)
        ctx.h, ctx.scale = H, float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        from . import _ext
        qkv, o, lse = ctx.saved_tensors
        B, N, _ = qkv.shape
        do = do.to(qkv.dtype).contiguous()
        dsum = torch.empty_like(lse)
        dqkv = torch.empty_like(qkv)
        _ext.call("mda_attn_bwd", qkv, o, do, lse, dsum, dqkv, B, N, ctx.h, ctx.scale)
        return dqkv, None, None


def attention_ref(qkv: torch.Tensor, num_heads: int, scale: float | None = None) -> torch.Tensor:
    B, N, C3 = qkv.shape
    D = C3 // (3 * num_heads)
    q, k, v = qkv.reshape(B, N, 3, num_heads, D).permute(2, 0, 3, 1, 4).unbind(0)
    out = F.scaled_dot_product_attention(q, k, v, scale=scale)
    return out.transpose(1, 2).reshape(B, N, num_heads * D)


def attention(qkv: torch.Tensor, num_heads: int, scale: float | None = None) -> torch.Tensor:
    D = qkv.shape[-1] // (3 * num_heads)
    scale = D ** -0.5 if scale is None else scale
    if native_ok(qkv, num_heads):
        return _FlashAttention.apply(qkv, num_heads, scale)
    return attention_ref(qkv, num_heads, scale)
