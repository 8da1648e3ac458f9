"""Contrastive Representation Distillation (reference `distillers/CRD.py:9-281`).

Student/teacher pooled features -> ``Embed`` (Linear + L2 norm) -> NCE
scores against K+1 rows of two momentum memory banks (the positive is the
sample's own row) -> ``ContrastLoss`` for both directions.

MI355X design:

* the gathered score / gradient passes are HIP kernels streaming bank rows
  (``ops/crd.py``); the B x (K+1) x D gather is never materialised;
* the normalisation constants Z live on device and are initialised without a
  host round trip; under data parallelism they are averaged across ranks on
  the first step so every replica normalises identically;
* memory updates are exchanged, not broadcast: every rank all-gathers the
  (index, v_s, v_t) rows of the global batch and applies all of them, so the
  banks stay bit-identical across ranks at B_global x (1 + 2D) floats per
  step.  The reference's DDP instead re-broadcasts the whole bank from rank 0
  every forward (48.8 MB CIFAR / 1.25 GB ImageNet) and drops the other
  ranks' updates.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.distributed as dist

from ._base import Distiller
from ..ops import crd as CO
from ..ops import losses as L


def _capturing(device=None) -> bool:
    if device is not None and torch.device(device).type != "cuda":
        return False
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class Normalize(nn.Module):
    def __init__(self, power=2):
        super().__init__()
        self.power = power

    def forward(self, x):
        norm = x.pow(self.power).sum(1, keepdim=True).pow(1.0 / self.power)
        return x.div(norm)


class _EmbedFn(torch.autograd.Function):
    """``l2norm(x W^T + b)`` on csrc/embed.hip: one launch forward, two
    backward (dgamma-style accumulation of dW / db straight into bound flat
    gradients), instead of the linear + normalise chain and its autograd."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from ..ops import _ext
        x = x.contiguous()
        N, K = x.shape
        D = weight.shape[0]
        out = torch.empty(N, D, dtype=torch.float32, device=x.device)
        norm = torch.empty(N, dtype=torch.float32, device=x.device)
        _ext.call("mda_embed_fwd", x, weight.detach(), bias.detach() if bias is not None else None,
                  out, norm, N, K, D)
        ctx.save_for_backward(x, weight, bias, out, norm)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..ops import _ext
        from ..parallel.grad_reducer import notify_grad
        x, weight, bias, out, norm = ctx.saved_tensors
        N, K = x.shape
        D = weight.shape[0]
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[2]
        direct = (need_w and weight.grad is not None and weight.grad.is_contiguous()
                  and (not need_b or bias.grad is not None))
        # the kernel computes db in the same pass as dW: a bias-only gradient
        # still needs a (scratch) dW target, or db would silently stay zero
        dw = weight.grad if direct else (torch.zeros_like(weight) if (need_w or need_b) else None)
        db = (bias.grad if direct else torch.zeros_like(bias)) if need_b else None
        dx = torch.empty_like(x) if need_x else None
        dy = torch.empty(N, D, dtype=torch.float32, device=x.device)
        _ext.call("mda_embed_bwd", dout.float().contiguous(), out, norm, x, weight.detach(), dy, dx,
                  dw, db, N, K, D)
        if direct:
            notify_grad(weight, *([bias] if need_b else []))
            return dx, None, None
        return dx, dw if need_w else None, db


class Embed(nn.Module):
    def __init__(self, dim_in=1024, dim_out=128):
        super().__init__()
        self.linear = nn.Linear(dim_in, dim_out)
        self.l2norm = Normalize(2)

    def forward(self, x):
        x = x.reshape(x.shape[0], -1).float()
        from ..ops.backend import hip_enabled_for
        if (hip_enabled_for(x) and x.shape[1] <= 2048 and x.shape[1] % 4 == 0
                and self.linear.out_features <= 1024):
            return _EmbedFn.apply(x, self.linear.weight, self.linear.bias)
        return self.l2norm(nn.functional.linear(x, self.linear.weight, self.linear.bias))


class ContrastLoss(nn.Module):
    """NCE loss with a uniform noise distribution (`CRD.py:116-141`)."""

    def __init__(self, num_data):
        super().__init__()
        self.num_data = num_data

    def forward(self, x):
        eps = 1e-7
        bsz = x.shape[0]
        m = x.size(1) - 1
        c = m / float(self.num_data)
        p_pos = x[:, 0]
        log_d1 = torch.log(p_pos / (p_pos + c + eps))
        p_neg = x[:, 1:]
        log_d0 = torch.log(c / (p_neg + c + eps))
        return -(log_d1.sum() + log_d0.sum()) / bsz


class ContrastMemory(nn.Module):
    """Two momentum memory banks + NCE normalisation constants (`CRD.py:144-220`).

    ``params`` = [K, T, Z_v1, Z_v2, momentum] (same buffer layout as the
    reference, so checkpoints carry the constants).
    """

    def __init__(self, input_size, output_size, K, T=0.07, momentum=0.5):
        super().__init__()
        self.n_lem = output_size
        self.K = int(K)
        self.T = float(T)
        self.momentum = float(momentum)
        self.register_buffer("params", torch.tensor([K, T, -1.0, -1.0, momentum]))
        stdv = 1.0 / math.sqrt(input_size / 3)
        self.register_buffer("memory_v1", torch.rand(output_size, input_size).mul_(2 * stdv).add_(-stdv))
        self.register_buffer("memory_v2", torch.rand(output_size, input_size).mul_(2 * stdv).add_(-stdv))
        self._z_ready = False

    def _init_z(self, out_v1, out_v2):
        z = torch.stack([out_v1.detach().mean(), out_v2.detach().mean()]) * self.n_lem
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(z)
            z /= dist.get_world_size()
        cur = self.params[2:4]
        self.params[2:4] = torch.where(cur < 0, z.to(cur.dtype), cur)
        self._z_ready = True

    def forward(self, v1, v2, y, idx):
        if idx is None:
            idx = torch.randint(0, self.n_lem, (v1.shape[0], self.K + 1), device=v1.device)
            idx[:, 0] = y
        out_v2 = CO.scores(self.memory_v1, idx, v2, self.T)
        out_v1 = CO.scores(self.memory_v2, idx, v1, self.T)
        if not self._z_ready:
            if float(self.params[2]) < 0 or float(self.params[3]) < 0:
                self._init_z(out_v1, out_v2)
            self._z_ready = True
        out_v1 = out_v1 / self.params[2]
        out_v2 = out_v2 / self.params[3]
        # the bank update is applied after backward (post_backward) so the
        # gradient sees the same rows as the forward, exactly as the
        # reference's detached index_select copy does
        self._pending = (v1.detach(), v2.detach(), y)
        return out_v1, out_v2

    def apply_pending(self):
        """After backward: world 1 applies the bank update; world > 1 packs the
        rank's (index, v1, v2) rows into a persistent buffer for
        :meth:`exchange` (eager, between the captured graphs) and
        :meth:`apply_exchange` (inside the update graph)."""
        pend = getattr(self, "_pending", None)
        if pend is None:
            return
        self._pending = None
        v1, v2, y = pend
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            self.update(v1, v2, y)
            return
        ws = dist.get_world_size()
        B, D = v1.shape
        # one (local, gathered) buffer pair PER batch shape, never rebound: the
        # captured fwd+bwd / update graphs keep the full-batch pair, and an eager
        # partial batch (the epoch's last, drop_last=False) gets its own pair
        # instead of freeing the memory those graphs were recorded against
        key = (B, D, v1.device)
        bufs = self.__dict__.setdefault("_xbufs", {})
        if key not in bufs:
            if _capturing(v1.device):
                raise RuntimeError("CRD exchange buffers must exist before capture "
                                   "(the eager warm-up step of the same shape creates them)")
            bufs[key] = (torch.empty(B, 1 + 2 * D, dtype=torch.float64, device=v1.device),
                         torch.empty(ws * B, 1 + 2 * D, dtype=torch.float64, device=v1.device))
        xl, _ = bufs[key]
        xl[:, 0].copy_(y)
        xl[:, 1:1 + D].copy_(v1)
        xl[:, 1 + D:].copy_(v2)
        if _capturing(v1.device):
            self._graph_key = key   # what every replay of the captured step staged into
        else:
            self._eager_key = key   # this eager step's rows (consumed by apply_exchange)

    def _xkey(self):
        """Buffers of the current step: an eager step's own pair, else the pair
        the captured graphs stage into (a replay runs no Python in between)."""
        k = None if _capturing() else self.__dict__.get("_eager_key")
        return k if k is not None else self.__dict__.get("_graph_key")

    def exchange(self):
        """The memory-update all-gather (a collective: never inside a capture
        in split mode; TrainStep calls it between the graphs)."""
        k = self._xkey()
        if k is not None:
            xl, xa = self._xbufs[k]
            dist.all_gather_into_tensor(xa, xl)

    @torch.no_grad()
    def apply_exchange(self):
        k = self._xkey()
        if k is None:
            return
        if not _capturing():
            self._eager_key = None
        _, xa = self._xbufs[k]
        D = k[1]
        y = xa[:, 0].long()
        CO.update(self.memory_v1, y, xa[:, 1:1 + D].float(), self.momentum)
        CO.update(self.memory_v2, y, xa[:, 1 + D:].float(), self.momentum)

    @torch.no_grad()
    def update(self, v1, v2, y):
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            ws = dist.get_world_size()
            packed = torch.cat([y.double().reshape(-1, 1), v1.double(), v2.double()], 1)
            allp = [torch.empty_like(packed) for _ in range(ws)]
            dist.all_gather(allp, packed)
            packed = torch.cat(allp, 0)
            D = v1.shape[1]
            y = packed[:, 0].long()
            v1 = packed[:, 1:1 + D].float()
            v2 = packed[:, 1 + D:].float()
        CO.update(self.memory_v1, y, v1, self.momentum)
        CO.update(self.memory_v2, y, v2, self.momentum)


class CRD(Distiller):
    teacher_needs = ("pooled",)
    # the memory-update exchange runs between the captured graphs (exchange /
    # apply_exchange), so CRD keeps hipGraphs at world > 1

    def __init__(self, student, teacher, cfg, num_data):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.CRD.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.CRD.LOSS.FEAT_WEIGHT
        self.embed_s = Embed(cfg.CRD.FEAT.STUDENT_DIM, cfg.CRD.FEAT.DIM)
        self.embed_t = Embed(cfg.CRD.FEAT.TEACHER_DIM, cfg.CRD.FEAT.DIM)
        self.contrast = ContrastMemory(cfg.CRD.FEAT.DIM, num_data, cfg.CRD.NCE.K,
                                       cfg.CRD.NCE.TEMPERATURE, cfg.CRD.NCE.MOMENTUM)
        self.criterion_s = ContrastLoss(num_data)
        self.criterion_t = ContrastLoss(num_data)

    def get_extra_parameters(self) -> int:
        n = sum(p.numel() for m in (self.embed_s, self.embed_t) for p in m.parameters())
        return n + sum(b.numel() for b in self.contrast.buffers())

    def post_backward(self):
        """Apply (world 1) or stage (world > 1) this step's memory-bank update
        (called by the trainer after backward)."""
        self.contrast.apply_pending()

    def exchange(self):
        """world > 1: all-gather the staged updates (eager, between graphs)."""
        self.contrast.exchange()

    def apply_exchange(self):
        """world > 1: apply every rank's update in rank order (in the update graph)."""
        self.contrast.apply_exchange()

    def crd_loss(self, f_s, f_t, idx, contrast_idx):
        f_s = self.embed_s(f_s)
        f_t = self.embed_t(f_t)
        out_s, out_t = self.contrast(f_s, f_t, idx, contrast_idx)
        return self.criterion_s(out_s) + self.criterion_t(out_t)

    def forward_train(self, image, target, index=None, contrastive_index=None, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        if index is None:
            raise ValueError("CRD needs the dataset index of every sample (CRD trainer)")
        loss_crd = self.feat_loss_weight * self.crd_loss(
            feature_student["pooled_feat"], feature_teacher["pooled_feat"], index, contrastive_index)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_crd}
