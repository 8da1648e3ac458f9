"""CRD memory-bank ops: gathered contrastive scores and momentum update.

HIP path: ``csrc/crd.hip`` (rows streamed from the bank, never materialised
as the reference's B x (K+1) x D gather).  PyTorch reference: the
reference's ``index_select`` + ``bmm`` (`distillers/CRD.py:164-220`).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from .backend import hip_enabled_for


def scores_ref(memory, idx, v, T):
    B, K1 = idx.shape
    w = torch.index_select(memory, 0, idx.reshape(-1)).detach().reshape(B, K1, -1)
    return torch.exp(torch.bmm(w, v.float().reshape(B, -1, 1)).squeeze(2) / T)


class _Scores(torch.autograd.Function):
    @staticmethod
    def forward(ctx, memory, idx, v, T):
        B, K1 = idx.shape
        D = memory.shape[1]
        v = v.float().contiguous()
        idx = idx.contiguous()
        e = torch.empty(B, K1, dtype=torch.float32, device=v.device)
        _ext.call("mda_crd_scores", memory, idx, v, e, B, K1, D, 1.0 / T)
        ctx.save_for_backward(memory, idx, e)
        ctx.T = T
        return e

    @staticmethod
    def backward(ctx, g):
        memory, idx, e = ctx.saved_tensors
        B, K1 = idx.shape
        D = memory.shape[1]
        g = g.float().contiguous()
        part = torch.empty(B * 16 * D, dtype=torch.float32, device=g.device)
        gv = torch.empty(B, D, dtype=torch.float32, device=g.device)
        _ext.call("mda_crd_grad", memory, idx, g, e, part, gv, B, K1, D, 1.0 / ctx.T)
        return None, None, gv, None


def scores(memory, idx, v, T):
    """``exp(<memory[idx[b,k]], v[b]> / T)``, shape (B, K+1); grad flows to ``v`` only."""
    if hip_enabled_for(v) and memory.dtype == torch.float32 and memory.shape[1] in (64, 128, 256):
        return _Scores.apply(memory, idx, v, float(T))
    return scores_ref(memory, idx, v, T)


@torch.no_grad()
def update_ref(memory, y, v, momentum):
    l = torch.index_select(memory, 0, y.reshape(-1)) * momentum + v.float() * (1 - momentum)
    memory.index_copy_(0, y, l / l.pow(2).sum(1, keepdim=True).sqrt())


@torch.no_grad()
def update(memory, y, v, momentum):
    """``memory[y] = normalize(m * memory[y] + (1 - m) * v)`` (rows of y unique)."""
    if hip_enabled_for(memory):
        _ext.call("mda_crd_update", memory, y.contiguous(), v.float().contiguous(), y.numel(),
                  memory.shape[1], float(momentum))
    else:
        update_ref(memory, y, v, momentum)
