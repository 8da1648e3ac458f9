"""Flat-buffer optimizers: SGD, Adam, AdamW and DOT (dual-momentum SGD).

Every learnable tensor of the distiller becomes a view into one contiguous
fp32 buffer (:class:`FlatParams`), and every ``.grad`` a view into a matching
flat gradient buffer.  Consequences:

* the data-parallel all-reduce is one (or a few bucketed) collective(s) on a
  contiguous buffer -- no per-tensor packing (:mod:`..parallel.grad_reducer`);
* each optimizer update is ONE fused HIP launch over the whole buffer
  (``csrc/optim.hip``) instead of a Python loop over tensors;
* the learning rate, the clip norm and the Adam step count live in device
  memory, so a captured hipGraph replays the step with new values.

The update rules are those of the reference (`engine/trainer.py:83-110`:
torch SGD/Adam/AdamW; `engine/dot.py:15-174`: DOT).  A pure-PyTorch
implementation of the same flat math serves CPU runs and is the numerical
reference the HIP kernels are tested against.

DOT keeps two gradient sets (task/CE and KD) in the two halves of one
``[2, n]`` buffer so both are all-reduced by a single collective -- the
reference's DDP reduces only the first backward.
"""
from __future__ import annotations

import math

import torch

from ..ops import _ext
from ..ops.backend import hip_enabled_for

ALIGN = 64  # elements (256 B): every view starts on a float4/cache-line boundary


class FlatParams:
    """Pack ``params`` into one flat buffer; params/grads become views.

    ``num_grad_sets`` = 2 allocates a second gradient buffer (DOT).
    Layout order is REVERSED registration order, so gradients produced early
    in backward (head first) are contiguous at the front of the buffer and
    can be reduced bucket by bucket while backward continues.
    """

    def __init__(self, params, num_grad_sets: int = 1):
        params = [p for p in params]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        dev = uniq[0].device if uniq else torch.device("cpu")
        self.device = dev
        self.offsets = []
        off = 0
        order = list(reversed(range(len(uniq))))
        offs = [0] * len(uniq)
        for i in order:
            offs[i] = off
            off += ((uniq[i].numel() + ALIGN - 1) // ALIGN) * ALIGN
        self.offsets = offs
        self.numel = max(off, ALIGN)
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(num_grad_sets, self.numel, dtype=torch.float32, device=dev)
        self.num_grad_sets = num_grad_sets
        for p, o in zip(uniq, offs):
            n = p.numel()
            self.data[o:o + n].copy_(p.detach().reshape(-1).float())
            p.data = self.data[o:o + n].view_as(p)
        self.bind_grads(0)

    @property
    def grad(self) -> torch.Tensor:
        return self.grads[0]

    def bind_grads(self, k: int) -> None:
        """Point every ``p.grad`` at gradient set ``k``."""
        g = self.grads[k]
        for p, o in zip(self.params, self.offsets):
            p.grad = g[o:o + p.numel()].view_as(p)
        self._bound = k

    def zero_grad(self) -> None:
        self.grads.zero_()

    def segment(self, p):
        i = next(j for j, q in enumerate(self.params) if q is p)
        return self.offsets[i], self.params[i].numel()

    def bucket_ranges(self, bucket_elems: int):
        """Contiguous ``[start, end)`` element ranges of the flat buffer."""
        ranges, start = [], 0
        while start < self.numel:
            end = min(self.numel, start + max(ALIGN, bucket_elems))
            ranges.append((start, end))
            start = end
        return ranges


class FlatOptimizer:
    """Base: holds lr/clip state on device and the fused/torch dispatch."""

    def __init__(self, flat: FlatParams, lr: float, weight_decay: float, grad_clip: float = 0.0,
                 grad_scale: float = 1.0):
        self.flat = flat
        dev = flat.device
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self._lr = float(lr)
        self.weight_decay = float(weight_decay)
        self.grad_clip = float(grad_clip)
        self.grad_scale = float(grad_scale)
        self.norm_t = torch.zeros(1, dtype=torch.float32, device=dev)
        self._norm_ws = torch.zeros(512, dtype=torch.float32, device=dev)
        self._norm_cnt = torch.zeros(4, dtype=torch.int32, device=dev)
        self.use_hip = hip_enabled_for(flat.data)
        self.param_groups = [{"lr": float(lr)}]  # torch-optimizer-like surface for schedulers

    # lr --------------------------------------------------------------------
    @property
    def lr(self) -> float:
        return self._lr

    def set_lr(self, lr: float) -> None:
        lr = float(lr)
        if lr != self._lr:
            self._lr = lr
            self.lr_t.fill_(lr)
        self.param_groups[0]["lr"] = lr

    # clip ------------------------------------------------------------------
    def _grad_norm(self, g: torch.Tensor):
        """Writes ||grad_scale * g|| into ``norm_t`` (device), returns it."""
        if self.use_hip:
            _ext.call("mda_sq_norm", g, g.numel(), self._norm_ws, self._norm_cnt, self.norm_t,
                      self.grad_scale)
        else:
            self.norm_t.copy_((g.double().pow(2).sum().sqrt() * self.grad_scale).float().reshape(1))
        return self.norm_t

    def _clip_coef_torch(self):
        if self.grad_clip <= 0:
            return 1.0
        return torch.clamp(self.grad_clip / (self.norm_t + 1e-6), max=1.0)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.flat.zero_grad()

    # parameters without a gradient ------------------------------------------
    def set_active(self, active) -> None:
        """``active``: per-param booleans (flat.params order).  torch.optim
        skips a parameter whose ``.grad`` is None -- no weight decay, no
        momentum -- so the update runs only over the flat ranges of params
        that receive a gradient (usually all: one launch)."""
        f = self.flat
        if all(active):
            self._ranges = None
            return
        segs = sorted((o, o + ((p.numel() + ALIGN - 1) // ALIGN) * ALIGN)
                      for p, o, a in zip(f.params, f.offsets, active) if a)
        ranges = []
        for s_, e_ in segs:
            if ranges and ranges[-1][1] == s_:
                ranges[-1][1] = e_
            else:
                ranges.append([s_, e_])
        self._ranges = [tuple(r) for r in ranges]

    def _spans(self):
        r = getattr(self, "_ranges", None)
        return [(0, self.flat.numel)] if r is None else r

    # torch.optim-format state (checkpoint compatibility with the reference) --
    def _unflatten(self, buf: torch.Tensor):
        f = self.flat
        return [buf[o:o + p.numel()].view_as(p).detach().clone().cpu() for p, o in zip(f.params, f.offsets)]

    def _flatten_into(self, buf: torch.Tensor, tensors) -> None:
        f = self.flat
        for p, o, t in zip(f.params, f.offsets, tensors):
            if t is not None:
                buf[o:o + p.numel()].copy_(t.reshape(-1).to(buf.device, buf.dtype))

    def _group(self, **extra) -> dict:
        g = {"lr": self._lr, "weight_decay": self.weight_decay,
             "params": list(range(len(self.flat.params)))}
        g.update(extra)
        return g

    @staticmethod
    def _per_param(sd: dict, key: str, n: int):
        st = sd.get("state", {})
        return [st.get(i, st.get(str(i), {})).get(key) for i in range(n)]

    def state_dict(self) -> dict:
        raise NotImplementedError

    def load_state_dict(self, sd: dict) -> None:
        raise NotImplementedError


class FlatSGD(FlatOptimizer):
    def __init__(self, flat, lr, momentum=0.9, weight_decay=0.0, grad_clip=0.0, grad_scale=1.0):
        super().__init__(flat, lr, weight_decay, grad_clip, grad_scale)
        self.momentum = float(momentum)
        self.buf = torch.zeros_like(flat.data)

    @torch.no_grad()
    def step(self) -> None:
        f = self.flat
        g = f.grads[0]
        norm = None
        if self.grad_clip > 0:
            norm = self._grad_norm(g)
        for a, b in self._spans():
            p_, g_, m_ = f.data[a:b], g[a:b], self.buf[a:b]
            if self.use_hip:
                _ext.call("mda_sgd_step", p_, g_, m_, self.lr_t, self.momentum,
                          self.weight_decay, self.grad_scale, norm, self.grad_clip, b - a)
                continue
            s = self.grad_scale * self._clip_coef_torch()
            d = g_ * s + self.weight_decay * p_
            if self.momentum != 0:
                m_.mul_(self.momentum).add_(d)
                d = m_
            p_.sub_(self.lr_t * d)

    def state_dict(self):
        bufs = self._unflatten(self.buf)
        return {"state": {i: {"momentum_buffer": b} for i, b in enumerate(bufs)},
                "param_groups": [self._group(momentum=self.momentum, dampening=0, nesterov=False,
                                             maximize=False)]}

    def load_state_dict(self, sd):
        self._flatten_into(self.buf, self._per_param(sd, "momentum_buffer", len(self.flat.params)))


class FlatAdam(FlatOptimizer):
    """torch.optim.Adam (``decoupled=False``) / AdamW (``decoupled=True``)."""

    def __init__(self, flat, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 decoupled=False, grad_clip=0.0, grad_scale=1.0):
        super().__init__(flat, lr, weight_decay, grad_clip, grad_scale)
        self.b1, self.b2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        self.decoupled = bool(decoupled)
        self.m1 = torch.zeros_like(flat.data)
        self.m2 = torch.zeros_like(flat.data)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=flat.device)

    @torch.no_grad()
    def step(self) -> None:
        f = self.flat
        g = f.grads[0]
        norm = self._grad_norm(g) if self.grad_clip > 0 else None
        self.step_t.add_(1.0)
        for a, b in self._spans():
            p_, g_, m1, m2 = f.data[a:b], g[a:b], self.m1[a:b], self.m2[a:b]
            if self.use_hip:
                _ext.call("mda_adam_step", p_, g_, m1, m2, self.lr_t, self.step_t,
                          self.b1, self.b2, self.eps, self.weight_decay, int(self.decoupled),
                          self.grad_scale, norm, self.grad_clip, b - a)
                continue
            s = self.grad_scale * self._clip_coef_torch()
            gv = g_ * s
            lr = self.lr_t
            if self.decoupled:
                p_.mul_(1 - lr * self.weight_decay)
            else:
                gv = gv + self.weight_decay * p_
            m1.mul_(self.b1).add_((1 - self.b1) * gv)
            m2.mul_(self.b2).add_((1 - self.b2) * gv * gv)
            t = self.step_t
            bc1 = 1 - torch.pow(torch.tensor(self.b1, device=t.device), t)
            bc2 = 1 - torch.pow(torch.tensor(self.b2, device=t.device), t)
            denom = m2.sqrt() / bc2.sqrt() + self.eps
            p_.sub_((lr / bc1) * m1 / denom)

    def state_dict(self):
        m1, m2 = self._unflatten(self.m1), self._unflatten(self.m2)
        step = self.step_t.detach().cpu().reshape(())
        return {"state": {i: {"step": step.clone(), "exp_avg": a, "exp_avg_sq": b}
                          for i, (a, b) in enumerate(zip(m1, m2))},
                "param_groups": [self._group(betas=(self.b1, self.b2), eps=self.eps, amsgrad=False,
                                             maximize=False)]}

    def load_state_dict(self, sd):
        n = len(self.flat.params)
        self._flatten_into(self.m1, self._per_param(sd, "exp_avg", n))
        self._flatten_into(self.m2, self._per_param(sd, "exp_avg_sq", n))
        steps = [s_ for s_ in self._per_param(sd, "step", n) if s_ is not None]
        if steps:
            self.step_t.fill_(float(torch.as_tensor(steps[0])))


class FlatDOT(FlatOptimizer):
    """Distillation-Oriented Trainer (reference `engine/dot.py:58-174`).

    Gradient set 0 = task (CE) grads, set 1 = KD grads.  ``mask`` (uint8 per
    element): bit0 = the element receives a task gradient, bit1 = a KD
    gradient; it is derived once from autograd reachability
    (:meth:`set_reachability`) because the reference's branches depend on
    which parameters have a ``.grad``.
    """

    def __init__(self, flat, lr, momentum, momentum_kd, weight_decay=0.0, grad_scale=1.0):
        assert flat.num_grad_sets == 2, "DOT needs FlatParams(num_grad_sets=2)"
        super().__init__(flat, lr, weight_decay, 0.0, grad_scale)
        self.mu_t = float(momentum)
        self.mu_k = float(momentum_kd)
        self.buf_t = torch.zeros_like(flat.data)
        self.buf_k = torch.zeros_like(flat.data)
        self.mask = torch.full((flat.numel,), 3, dtype=torch.uint8, device=flat.device)
        self.first = True

    def set_reachability(self, has_task, has_kd) -> None:
        """``has_task``/``has_kd``: per-param booleans (same order as flat.params)."""
        m = torch.zeros(self.flat.numel, dtype=torch.uint8)
        for p, o, t, k in zip(self.flat.params, self.flat.offsets, has_task, has_kd):
            m[o:o + p.numel()] = (1 if t else 0) | (2 if k else 0)
        self.mask.copy_(m.to(self.mask.device))

    @torch.no_grad()
    def step(self) -> None:
        f = self.flat
        gt, gk = f.grads[0], f.grads[1]
        if self.use_hip:
            _ext.call("mda_dot_step", f.data, gt, gk, self.buf_t, self.buf_k, self.mask, self.lr_t,
                      self.mu_t, self.mu_k, self.weight_decay, self.grad_scale, int(self.first),
                      f.numel)
        else:
            self._step_torch(gt, gk)
        self.first = False

    def _step_torch(self, gt, gk):
        f, s, wd = self.flat, self.grad_scale, self.weight_decay
        has_t = (self.mask & 1).bool()
        has_k = (self.mask & 2).bool()
        mu_avg = 0.5 * (self.mu_t + self.mu_k)
        lr = self.lr_t
        p = f.data
        d = s * gt + wd * p
        if self.first:
            bt = d
        else:
            bt = torch.where(has_k, self.mu_t, mu_avg) * self.buf_t + d
        self.buf_t.copy_(torch.where(has_t, bt, self.buf_t))
        p.sub_(torch.where(has_t, lr * self.buf_t, torch.zeros_like(p)))
        dk = s * gk
        if self.first:
            bk = dk
        else:
            bk = torch.where(has_t, self.mu_k * self.buf_k + dk, mu_avg * self.buf_k + dk + wd * p)
        self.buf_k.copy_(torch.where(has_k, bk, self.buf_k))
        p.sub_(torch.where(has_k, lr * self.buf_k, torch.zeros_like(p)))

    def state_dict(self):
        bt, bk = self._unflatten(self.buf_t), self._unflatten(self.buf_k)
        return {"state": {i: {"momentum_buffer": a, "momentum_kd_buffer": b}
                          for i, (a, b) in enumerate(zip(bt, bk))},
                "param_groups": [self._group(momentum=self.mu_t, momentum_kd=self.mu_k, dampening=0)],
                "mda_dot": {"mask": self.mask.detach().cpu().clone(), "first": self.first}}

    def load_state_dict(self, sd):
        n = len(self.flat.params)
        self._flatten_into(self.buf_t, self._per_param(sd, "momentum_buffer", n))
        self._flatten_into(self.buf_k, self._per_param(sd, "momentum_kd_buffer", n))
        extra = sd.get("mda_dot")
        if extra is not None:
            self.mask.copy_(extra["mask"].to(self.mask.device))
            self.first = bool(extra["first"])
        else:
            self.first = False


def build_optimizer(cfg, flat: FlatParams, grad_scale: float = 1.0, trainer: str = "base"):
    """Optimizer from the cfg (reference `trainer.py:83-110`, DOT `:376-391`)."""
    lr = cfg.SOLVER.LR
    wd = cfg.SOLVER.WEIGHT_DECAY
    clip = float(cfg.SOLVER.GRAD_CLIP)
    if trainer in ("dot", "crd_dot"):
        mu = cfg.SOLVER.SGD.MOMENTUM
        delta = cfg.SOLVER.DOT.DELTA
        return FlatDOT(flat, lr, momentum=mu - delta, momentum_kd=mu + delta, weight_decay=wd,
                       grad_scale=grad_scale)
    typ = cfg.SOLVER.TYPE.upper()
    if typ == "SGD":
        return FlatSGD(flat, lr, momentum=cfg.SOLVER.SGD.MOMENTUM, weight_decay=wd,
                       grad_clip=clip, grad_scale=grad_scale)
    if typ in ("ADAM", "ADAMW"):
        return FlatAdam(flat, lr, betas=tuple(cfg.SOLVER.ADAM.BETAS), eps=cfg.SOLVER.ADAM.EPSILON,
                        weight_decay=wd, decoupled=(typ == "ADAMW"), grad_clip=clip,
                        grad_scale=grad_scale)
    raise NotImplementedError(cfg.SOLVER.TYPE)
