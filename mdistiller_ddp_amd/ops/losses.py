"""Logit-distillation losses: CE, KD, DKD.

Each loss has a plain-PyTorch reference (a direct transcription of the
reference formulas: `distillers/KD.py:8-13`, `distillers/DKD.py:8-51`) and a
fused HIP path (``csrc/losses.hip``): one launch reads the student/teacher
logits once and produces both scalar losses and both gradients w.r.t. the
student logits; the autograd backward is a single ``axpby`` that scales the
stored gradients by the incoming loss gradients (device scalars, so it is
hipGraph-replay safe and works with the two-backward DOT trainer).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext
from .backend import hip_enabled_for

# --------------------------------------------------------------------------
# PyTorch references


def kd_loss_ref(logits_student, logits_teacher, temperature):
    log_pred_student = F.log_softmax(logits_student.float() / temperature, dim=1)
    pred_teacher = F.softmax(logits_teacher.float() / temperature, dim=1)
    loss = F.kl_div(log_pred_student, pred_teacher, reduction="none").sum(1).mean()
    return loss * temperature ** 2


def _gt_mask(logits, target):
    return torch.zeros_like(logits, dtype=torch.bool).scatter_(1, target.reshape(-1, 1), True)


def dkd_loss_ref(logits_student, logits_teacher, target, alpha, beta, temperature):
    s = logits_student.float()
    t = logits_teacher.float()
    gt = _gt_mask(s, target)
    other = ~gt
    ps = F.softmax(s / temperature, dim=1)
    pt = F.softmax(t / temperature, dim=1)
    bs = torch.stack([(ps * gt).sum(1), (ps * other).sum(1)], dim=1)
    bt = torch.stack([(pt * gt).sum(1), (pt * other).sum(1)], dim=1)
    B = target.shape[0]
    tckd = F.kl_div(torch.log(bs), bt, reduction="sum") * temperature ** 2 / B
    pt2 = F.softmax(t / temperature - 1000.0 * gt, dim=1)
    ls2 = F.log_softmax(s / temperature - 1000.0 * gt, dim=1)
    nckd = F.kl_div(ls2, pt2, reduction="sum") * temperature ** 2 / B
    return alpha * tckd + beta * nckd


def cross_entropy(logits, target):
    return F.cross_entropy(logits.float(), target)


# --------------------------------------------------------------------------
# fused HIP path

_DT = {torch.float32: 0, torch.bfloat16: 1}
_MODES = {"ce": 0, "kd": 1, "dkd": 2}


class _Workspace:
    """Per-device scratch: partial sums + arrival counter (zeroed once)."""

    def __init__(self, device):
        self.partial = torch.zeros(4096, dtype=torch.float32, device=device)
        self.counter = torch.zeros(4, dtype=torch.int32, device=device)


_WS: dict = {}


def workspace(device) -> _Workspace:
    key = torch.device(device).index or 0
    ws = _WS.get(key)
    if ws is None:
        ws = _WS[key] = _Workspace(device)
    return ws


_UNIT_SEEDS: list = []   # strong references: their memory is never reused
_UNIT_PTRS: set = set()


def register_unit_seed(t: torch.Tensor) -> None:
    """``t`` is a scalar that holds 1.0 for as long as the process lives and is
    never written (the training step's backward seed, engine/step.py).  A
    logit-loss backward that receives it returns the stored gradient as is
    instead of launching the ``go * g`` scaling."""
    if t.numel() == 1 and t.data_ptr() not in _UNIT_PTRS:
        _UNIT_SEEDS.append(t)
        _UNIT_PTRS.add(t.data_ptr())


def _is_unit(go) -> bool:
    return go is not None and go.numel() == 1 and go.data_ptr() in _UNIT_PTRS


def _supported(s, t, C):
    return (s.dim() == 2 and s.dtype in _DT and (t is None or t.dtype in _DT)
            and C <= 2048 and s.shape[0] <= 8192)


class _LogitLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, t, target, mode, inv_T, ce_w, kd_w, alpha, beta, epoch=None, warmup=0.0):
        s = s.contiguous()
        t = s if t is None else t.contiguous()
        target = target.contiguous().to(torch.int64)
        B, C = s.shape
        g_ce = torch.empty_like(s)
        g_kd = torch.empty_like(s) if mode != 0 else g_ce
        # g_ce + g_kd for the unit-seed backward (not needed by DOT's stacked sets)
        from .hip_train import _DUAL
        g_sum = torch.empty_like(s) if (mode != 0 and _DUAL[0] is None) else None
        losses = torch.empty(2, dtype=torch.float32, device=s.device)
        ws = workspace(s.device)
        _ext.call("mda_logit_loss", mode, _DT[s.dtype], _DT[t.dtype], s, t, target, g_ce, g_kd,
                  ws.partial, ws.counter, losses, B, C, inv_T, ce_w, kd_w, alpha, beta,
                  _epoch_ptr(epoch, warmup), float(warmup or 0.0), g_sum)
        ctx.save_for_backward(g_ce, g_kd, g_sum)
        ctx.mode = mode
        # an unused loss output gets no zero-filled gradient (one launch less)
        ctx.set_materialize_grads(False)
        return losses[0], losses[1]

    @staticmethod
    def backward(ctx, go_ce, go_kd):
        g_ce, g_kd, g_sum = ctx.saved_tensors
        from .hip_train import _DUAL, dual_alloc
        if go_ce is None and go_kd is None:
            return (None,) * 11
        if _DUAL[0] is None:
            # the training step's constant unit seeds: nothing to scale
            uce, ukd = _is_unit(go_ce), _is_unit(go_kd)
            if ctx.mode == 0 or go_kd is None:
                if uce:
                    return (g_ce,) + (None,) * 10
            elif go_ce is None:
                if ukd:
                    return (g_kd,) + (None,) * 10
            elif uce and ukd and g_sum is not None:
                return (g_sum,) + (None,) * 10
        if _DUAL[0] is not None:
            # DOT single-pass backward: [go_kd * g_kd ; go_ce * g_ce] stacked,
            # the KD set first (ops/hip_train.py _Dual)
            if ctx.mode == 0 or go_ce is None or go_kd is None:
                raise RuntimeError("DOT single-pass backward needs both the CE and the KD loss")
            full, half = dual_alloc(tuple(g_ce.shape), g_ce.dtype, g_ce.device)
            B = g_ce.shape[0]
            n = g_ce.numel()
            _ext.call("mda_axpby", _DT[full.dtype], None, g_ce, go_kd.float().reshape(1).contiguous(),
                      g_kd, full[:B], n)
            _ext.call("mda_axpby", _DT[full.dtype], go_ce.float().reshape(1).contiguous(), g_ce,
                      None, g_kd, full[B:], n)
            return half, None, None, None, None, None, None, None, None, None, None
        out = torch.empty_like(g_ce)
        a = None if go_ce is None else go_ce.float().reshape(1).contiguous()
        b = None if (go_kd is None or ctx.mode == 0) else go_kd.float().reshape(1).contiguous()
        _ext.call("mda_axpby", _DT[out.dtype], a, g_ce, b, g_kd, out, out.numel())
        return out, None, None, None, None, None, None, None, None, None, None


def _epoch_ptr(epoch, warmup):
    """Device fp32 epoch scalar for the in-kernel warm-up factor, or None."""
    if epoch is None or not warmup or warmup <= 0:
        return None
    if not isinstance(epoch, torch.Tensor) or epoch.dtype != torch.float32 or not epoch.is_cuda:
        raise TypeError("warm-up epoch must be a float32 device tensor on the HIP path")
    return epoch


def ce_kd(logits_s, logits_t, target, temperature, ce_weight, kd_weight):
    """``(ce_weight * CE(s, y), kd_weight * KD_T(s, t))``."""
    C = logits_s.shape[1]
    if hip_enabled_for(logits_s) and _supported(logits_s, logits_t, C):
        return _LogitLoss.apply(logits_s, logits_t.detach(), target, 1, 1.0 / float(temperature),
                                float(ce_weight), float(kd_weight), 0.0, 0.0)
    return (ce_weight * cross_entropy(logits_s, target),
            kd_weight * kd_loss_ref(logits_s, logits_t.detach(), temperature))


def _warmup(epoch, warmup):
    if epoch is None or not warmup or warmup <= 0:
        return 1.0
    if isinstance(epoch, torch.Tensor):
        return torch.clamp(epoch.float() / float(warmup), max=1.0)
    return min(float(epoch) / float(warmup), 1.0)


def ce_dkd(logits_s, logits_t, target, ce_weight, alpha, beta, temperature, epoch=None, warmup=0):
    """``(ce_weight * CE(s, y), min(epoch / warmup, 1) * DKD(s, t))``.

    The warm-up factor (``DKD.WARMUP``, reference ``DKD.py:78``) is applied
    inside the fused kernel from the device epoch tensor when one is given.
    """
    C = logits_s.shape[1]
    if (hip_enabled_for(logits_s) and _supported(logits_s, logits_t, C)
            and (epoch is None or isinstance(epoch, torch.Tensor) or not warmup)):
        ep = epoch if isinstance(epoch, torch.Tensor) else None
        if ep is not None and (ep.dtype != torch.float32 or ep.device != logits_s.device):
            ep = ep.to(device=logits_s.device, dtype=torch.float32)
        return _LogitLoss.apply(logits_s, logits_t.detach(), target, 2, 1.0 / float(temperature),
                                float(ce_weight), 1.0, float(alpha), float(beta), ep,
                                float(warmup or 0.0) if ep is not None else 0.0)
    return (ce_weight * cross_entropy(logits_s, target),
            _warmup(epoch, warmup) * dkd_loss_ref(logits_s, logits_t.detach(), target, alpha, beta,
                                                  temperature))


def ce(logits_s, target, ce_weight=1.0):
    C = logits_s.shape[1]
    if hip_enabled_for(logits_s) and _supported(logits_s, None, C):
        return _LogitLoss.apply(logits_s, None, target, 0, 1.0, float(ce_weight), 0.0, 0.0, 0.0)[0]
    return ce_weight * cross_entropy(logits_s, target)


def kd_loss(logits_student, logits_teacher, temperature):
    return ce_kd(logits_student, logits_teacher, torch.zeros(logits_student.shape[0], dtype=torch.long,
                 device=logits_student.device), temperature, 0.0, 1.0)[1]


def dkd_loss(logits_student, logits_teacher, target, alpha, beta, temperature):
    return ce_dkd(logits_student, logits_teacher, target, 0.0, alpha, beta, temperature)[1]
