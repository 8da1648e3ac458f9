"""Functional layer ops used by every model in the zoo.

Models keep standard ``nn.Conv2d`` / ``nn.BatchNorm2d`` sub-modules (so their
``state_dict`` keys are identical to the reference checkpoints) but run their
forward through these functions.  Each function has two implementations:

* the PyTorch reference (CPU, tests, fallback for shapes the kernels do not
  cover), and
* the HIP path (``ops/hip_layers.py``): one MFMA implicit-GEMM launch per
  conv whose epilogue applies the folded BN affine + residual + activation in
  eval mode, or emits per-channel batch statistics in train mode.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .backend import hip_enabled_for

_ACTS = ("relu", "relu6", "none")
# training-mode native conv+BN path (ops/hip_train.py); switchable for A/B runs
_TRAIN_KERNELS = {"on": True}


def set_train_kernels(flag: bool) -> None:
    _TRAIN_KERNELS["on"] = bool(flag)


def activate(x: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return F.relu(x)
    if act == "relu6":
        return F.relu6(x)
    if act == "none":
        return x
    raise ValueError(act)


# Train-mode BatchNorms that ran WITHOUT autograd on the PyTorch/MIOpen path
# (e.g. a frozen teacher kept in train-mode BN by OFD whose layer the native
# no-grad kernels do not serve).  MIOpen's bf16 train-mode BN replayed from a
# hipGraph went non-finite (profiles/r1_ofd_graph_ab.md), so a distiller that
# captures such a teacher checks this counter after its eager warm-up.
_TRAINBN_FALLBACKS = {"n": 0}


def trainbn_fallbacks() -> int:
    return _TRAINBN_FALLBACKS["n"]


def _bn(x: torch.Tensor, bn: nn.BatchNorm2d) -> torch.Tensor:
    if bn.training and not torch.is_grad_enabled():
        _TRAINBN_FALLBACKS["n"] += 1
    return bn(x)


def conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d | None = None,
                act: str = "relu", residual: torch.Tensor | None = None,
                want_preact: bool = False, fork=None, res_fork=None, defer_apply: bool = False,
                private: bool = False):
    """``act(bn(conv(x)) + residual)``; returns ``(out, preact_or_None)``.

    ``fork`` / ``res_fork`` (:class:`ops.hip_train.GradFork`, optional): x /
    residual also feed another native layer; their gradients are summed
    inside the native backward (no autograd add) -- ignored off that path.
    ``defer_apply`` (a projection shortcut, ``act="none"``): on the native
    training path the BN apply is left to the one consumer, which must be a
    native conv + BN taking the result as ``residual``
    (:class:`ops.hip_train.VirtualBN`; see :func:`ops.hip_train.can_defer_residual`).
    ``private``: the output feeds only native convs / native residual consumers
    (no feature loss, no other autograd consumer), so the consuming conv's
    dgrad may finish this BN's backward in its own launch."""
    if hip_enabled_for(x):
        from . import hip_layers
        if hip_layers.conv_supported(x, conv, bn):
            return hip_layers.conv_bn_act(x, conv, bn, act, residual, want_preact)
        from . import hip_train
        if _TRAIN_KERNELS["on"] and hip_train.train_supported(x, conv, bn):
            return hip_train.conv_bn_act_train(x, conv, bn, act, residual, want_preact, fork,
                                               res_fork, defer_apply, private)
    if residual is not None and getattr(residual, "_mda_vbn", None) is not None:
        raise RuntimeError("a VirtualBN residual reached a non-native consumer "
                           "(check ops.hip_train.can_defer_residual at the call site)")
    if getattr(x, "_mda_vbn", None) is not None:
        raise RuntimeError("a virtual (un-applied) BN output reached a non-native consumer")
    if hip_enabled_for(x):
        from . import hip_train
        if _TRAIN_KERNELS["on"] and bn is None and hip_train.conv_train_supported(x, conv):
            return hip_train.conv_act_train(x, conv, act, residual, want_preact)
        if hip_train.trainbn_nograd_supported(x, conv, bn):
            return hip_train.conv_trainbn_nograd(x, conv, bn, act, residual, want_preact)
    # the raw convolution (not ``conv(x)``): modules that route their own
    # forward through this op -- e.g. the detection Conv2d with a norm child --
    # must not recurse
    y = nn.Conv2d._conv_forward(conv, x, conv.weight, conv.bias) if isinstance(conv, nn.Conv2d) else conv(x)
    if bn is not None and isinstance(bn, nn.BatchNorm2d) and hip_enabled_for(y):
        # convolution on PyTorch (grouped 1x1 of ShuffleNetV1, odd shapes), the
        # BN (+res) (+act) still on the fused native kernels
        return bn_act(y, bn, act, residual, want_preact)
    if bn is not None:
        y = _bn(y, bn)
    if residual is not None:
        y = y + residual
    out = activate(y, act)
    return out, (y if want_preact else None)


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, act: str = "relu",
           residual: torch.Tensor | None = None, want_preact: bool = False):
    """``act(bn(x) + residual)`` (pre-activation blocks, WRN/ResNet heads)."""
    if hip_enabled_for(x):
        from . import hip_layers
        if hip_layers.bn_supported(x, bn):
            return hip_layers.bn_act(x, bn, act, residual, want_preact)
        from . import hip_train
        if _TRAIN_KERNELS["on"] and hip_train.bn_train_supported(x, bn):
            return hip_train.bn_act_train(x, bn, act, residual, want_preact)
    y = _bn(x, bn)
    if residual is not None:
        y = y + residual
    out = activate(y, act)
    return out, (y if want_preact else None)


def conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    return conv_bn_act(x, conv, None, "none")[0]


class _ChannelShuffle(torch.autograd.Function):
    """NHWC bf16 channel shuffle in one gather pass (csrc/pool.hip); the
    backward is the inverse shuffle (groups' = C / groups)."""

    @staticmethod
    def forward(ctx, x, groups):
        from . import _ext
        x = x.contiguous(memory_format=torch.channels_last)
        n, c, h, w = x.shape
        y = torch.empty_like(x)
        _ext.call("mda_channel_shuffle", x, y, n * h * w, c, groups)
        ctx.groups = groups
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _ext
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, c, h, w = dy.shape
        dx = torch.empty_like(dy)
        _ext.call("mda_channel_shuffle", dy, dx, n * h * w, c, c // ctx.groups)
        return dx, None


class _ChannelGather(torch.autograd.Function):
    """y[:, c] = x[:, fmap[c]] (0 where fmap[c] < 0) on NHWC bf16 in one pass
    (csrc/pool.hip mda_channel_gather); backward = the same gather with the
    inverse map (the maps are injective)."""

    @staticmethod
    def forward(ctx, x, fmap, bmap):
        from . import _ext
        x = x.contiguous(memory_format=torch.channels_last)
        n, c, h, w = x.shape
        y = torch.empty((n, fmap.numel(), h, w), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        _ext.call("mda_channel_gather", x, y, fmap, n * h * w, c, fmap.numel())
        ctx.maps = (bmap, c)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _ext
        bmap, cx = ctx.maps
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, c, h, w = dy.shape
        dx = torch.empty((n, cx, h, w), dtype=dy.dtype, device=dy.device,
                         memory_format=torch.channels_last)
        _ext.call("mda_channel_gather", dy, dx, bmap, n * h * w, c, cx)
        return dx, None, None


def channel_gather(x: torch.Tensor, fmap: torch.Tensor, bmap: torch.Tensor) -> torch.Tensor:
    """Channel gather with zero fill: ``fmap`` (int32, one entry per output
    channel, -1 = zero) and its inverse ``bmap`` (one entry per input channel)."""
    if (hip_enabled_for(x) and x.dtype == torch.bfloat16 and fmap.numel() % 2 == 0
            and bmap.numel() % 2 == 0 and fmap.is_cuda):
        return _ChannelGather.apply(x, fmap, bmap)
    idx = fmap.long().clamp_min(0)
    y = x.index_select(1, idx)
    return y * (fmap >= 0).to(y.dtype).reshape(1, -1, 1, 1)


class _Gather2(torch.autograd.Function):
    """Up to two NHWC bf16 outputs gathered channel-wise from up to two
    sources (csrc/pool.hip mda_gather2): ``y_d[:, j] = src_{f_d[j] >> 16}[:,
    f_d[j] & 0xffff]`` (0 where f_d[j] < 0).  The maps are injective, so the
    backward is the same gather with the inverse maps ``b_s[c] = (d << 16) | j``
    -- one launch per source gradient, no autograd add."""

    @staticmethod
    def forward(ctx, x0, x1, fmaps, bmaps, couts):
        from . import _ext
        srcs = [t.contiguous(memory_format=torch.channels_last) for t in (x0, x1) if t is not None]
        a = srcs[0]
        b = srcs[1] if len(srcs) > 1 else srcs[0]
        n, _, h, w = a.shape
        ys = [torch.empty((n, c, h, w), dtype=torch.bfloat16, device=a.device,
                          memory_format=torch.channels_last) for c in couts]
        two = len(ys) > 1
        _ext.call("mda_gather2", a, b, ys[0], fmaps[0], couts[0], ys[1] if two else None,
                  fmaps[1] if two else None, couts[1] if two else 0, n * h * w, a.shape[1],
                  b.shape[1])
        ctx.meta = (bmaps, [t.shape[1] for t in srcs], couts, n, h, w)
        return tuple(ys) if two else ys[0]

    @staticmethod
    def backward(ctx, *dys):
        from . import _ext
        bmaps, cins, couts, n, h, w = ctx.meta
        dys = [d.to(torch.bfloat16).contiguous(memory_format=torch.channels_last) if d is not None
               else torch.zeros((n, c, h, w), dtype=torch.bfloat16, device=bmaps[0].device,
                                memory_format=torch.channels_last) for d, c in zip(dys, couts)]
        a = dys[0]
        b = dys[1] if len(dys) > 1 else dys[0]
        want = [k for k in range(len(cins)) if ctx.needs_input_grad[k]]
        grads = [None, None]
        if want:
            outs = [torch.empty((n, cins[k], h, w), dtype=torch.bfloat16, device=a.device,
                                memory_format=torch.channels_last) for k in want]
            two = len(want) > 1
            # both source gradients from both output gradients: one launch
            _ext.call("mda_gather2", a, b, outs[0], bmaps[want[0]], cins[want[0]],
                      outs[1] if two else None, bmaps[want[1]] if two else None,
                      cins[want[1]] if two else 0, n * h * w, a.shape[1], b.shape[1])
            for k, o in zip(want, outs):
                grads[k] = o
        return grads[0], grads[1], None, None, None


class ChannelRoute:
    """A fixed channel routing ``outputs[d][j] <- sources[s][c]`` (or zero) for
    :func:`gather2`: device maps for the HIP kernel + index maps for the
    PyTorch fallback.  ``routes``: per output, a list of (s, c) or None."""

    def __init__(self, routes, cins):
        self.cins = list(cins)
        self.couts = [len(r) for r in routes]
        enc = lambda sc: -1 if sc is None else (sc[0] << 16) | sc[1]  # noqa: E731
        self.f = [torch.tensor([enc(sc) for sc in r], dtype=torch.int32) for r in routes]
        inv = [[-1] * c for c in self.cins]
        for d, r in enumerate(routes):
            for j, sc in enumerate(r):
                if sc is not None:
                    if inv[sc[0]][sc[1]] != -1:
                        raise ValueError("ChannelRoute: a source channel is routed twice")
                    inv[sc[0]][sc[1]] = (d << 16) | j
        self.b = [torch.tensor(v, dtype=torch.int32) for v in inv]
        # fallback: index into cat(sources + [zero column])
        off = [0]
        for c in self.cins:
            off.append(off[-1] + c)
        self.idx = [torch.tensor([off[-1] if sc is None else off[sc[0]] + sc[1] for sc in r],
                                 dtype=torch.long) for r in routes]
        self._dev = {}

    def maps(self, device):
        key = str(device)
        v = self._dev.get(key)
        if v is None:
            v = self._dev[key] = ([t.to(device) for t in self.f], [t.to(device) for t in self.b],
                                  [t.to(device) for t in self.idx])
        return v


def gather2(route: ChannelRoute, x0, x1=None):
    """Apply ``route`` to the sources; returns one tensor or a tuple of two."""
    f, b, idx = route.maps(x0.device)
    srcs = [t for t in (x0, x1) if t is not None]
    if (hip_enabled_for(x0) and all(t.dtype == torch.bfloat16 for t in srcs)
            and all(c % 2 == 0 for c in route.couts + route.cins)
            and sum(route.couts) <= 4096 and sum(route.cins) <= 4096):
        return _Gather2.apply(x0, x1, f, b, route.couts)
    z = torch.zeros_like(srcs[0][:, :1])
    cat = torch.cat(srcs + [z], 1)
    ys = [cat.index_select(1, i) for i in idx]
    return tuple(ys) if len(ys) > 1 else ys[0]


class _ShuffleTail(torch.autograd.Function):
    """ShuffleNetV1 stride-2 unit tail ``pre = cat([y3, avgpool3x3s2(x)]);
    out = relu(pre)`` in one HIP pass, backward in one more (csrc/pool.hip).
    ``fork``: x also feeds conv1; the pooled path's gradient is parked and
    summed in conv1's dgrad epilogue (ops.hip_train.GradFork)."""

    @staticmethod
    def forward(ctx, y3, x, fork):
        from . import _ext
        ctx.set_materialize_grads(False)
        y3 = y3.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        N, C3, Ho, Wo = y3.shape
        _, Cx, H, W = x.shape
        pre = torch.empty((N, C3 + Cx, Ho, Wo), dtype=torch.bfloat16, device=x.device,
                          memory_format=torch.channels_last)
        out = torch.empty_like(pre)
        _ext.call("mda_shuffle_tail_fwd", y3, x, pre, out, N, H, W, Ho, Wo, C3, Cx)
        ctx.save_for_backward(pre)
        ctx.meta = (N, H, W, Ho, Wo, C3, Cx)
        ctx.fork = fork.join() if fork is not None else None
        return out, pre

    @staticmethod
    def backward(ctx, dout, dpre):
        from . import _ext
        from .hip_train import _fork_sum
        pre, = ctx.saved_tensors
        N, H, W, Ho, Wo, C3, Cx = ctx.meta
        cl = torch.channels_last
        if dout is None:
            dout = torch.zeros_like(pre)
        dout = dout.to(torch.bfloat16).contiguous(memory_format=cl)
        dpre = dpre.to(torch.bfloat16).contiguous(memory_format=cl) if dpre is not None else None
        dy3 = torch.empty((N, C3, Ho, Wo), dtype=torch.bfloat16, device=pre.device, memory_format=cl)
        dx = torch.empty((N, Cx, H, W), dtype=torch.bfloat16, device=pre.device, memory_format=cl)
        _ext.call("mda_shuffle_tail_bwd", dout, dpre, pre, dy3, dx, N, H, W, Ho, Wo, C3, Cx)
        return dy3, _fork_sum(ctx.fork, dx), None


def shuffle_tail(y3: torch.Tensor, x: torch.Tensor, fork=None):
    """``(relu(pre), pre)`` with ``pre = cat([y3, avg_pool2d(x, 3, 2, 1)], 1)``."""
    if (hip_enabled_for(x) and x.dim() == 4 and y3.shape[1] % 8 == 0 and x.shape[1] % 8 == 0
            and y3.shape[2] == (x.shape[2] + 1) // 2 and y3.shape[3] == (x.shape[3] + 1) // 2
            and x.dtype in (torch.bfloat16, torch.float32) and y3.dtype in (torch.bfloat16, torch.float32)):
        return _ShuffleTail.apply(y3, x, fork)
    pre = torch.cat([y3, F.avg_pool2d(x, 3, stride=2, padding=1).to(y3.dtype)], 1)
    return F.relu(pre), pre


def channel_shuffle(x: torch.Tensor, groups: int) -> torch.Tensor:
    n, c, h, w = x.shape
    if (hip_enabled_for(x) and x.dtype == torch.bfloat16 and c % groups == 0 and c % 2 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _ChannelShuffle.apply(x, groups)
    return x.reshape(n, groups, c // groups, h, w).transpose(1, 2).reshape(n, c, h, w)


def linear(x: torch.Tensor, fc: nn.Linear) -> torch.Tensor:
    return fc(x)


class _PoolFC(torch.autograd.Function):
    """Global average pool + Linear on the fused HIP head kernels (csrc/head.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import _ext
        N, C, H, W = x.shape
        J = weight.shape[0]
        ctx.set_materialize_grads(False)  # an unused pooled output gets no zero gradient
        dt = 0 if x.dtype == torch.float32 else 1
        xc = x.contiguous(memory_format=torch.channels_last)
        pooled = torch.empty(N, C, dtype=x.dtype, device=x.device)
        logits = torch.empty(N, J, dtype=x.dtype, device=x.device)
        w = weight.detach()
        b = bias.detach() if bias is not None else None
        _ext.call("mda_pool_fc_fwd", dt, xc, w, b, pooled, logits, N, H * W, C, J)
        ctx.save_for_backward(pooled, weight, bias)
        ctx.meta = (N, C, H, W, J, dt, bias is not None)
        # x is a training BN's output (hip_train.BnLink): the backward's dx is
        # that layer's whole output gradient, so the head kernel also adds its
        # backward sums (small bf16 heads only; see csrc/head.hip)
        from .hip_train import _BNB_ON
        link = getattr(x, "_mda_bnlink", None) if _BNB_ON[0] else None
        ctx.link = link if (link is not None and dt == 1 and J * C <= (1 << 16) and C <= 2048
                            and link.C == C and link.M == N * H * W) else None
        return pooled, logits

    @staticmethod
    def backward(ctx, dpooled, dlogits):
        from . import _ext
        from .hip_train import _DUAL
        if _DUAL[0] is not None:
            return _PoolFC._backward_dual(ctx, dpooled, dlogits)
        pooled, weight, bias = ctx.saved_tensors
        N, C, H, W, J, dt, has_b = ctx.meta
        dev = pooled.device
        dtype = pooled.dtype
        if dlogits is None:
            dlogits = torch.zeros(N, J, dtype=dtype, device=dev)
        dlogits = dlogits.to(dtype).contiguous()
        dpooled = dpooled.to(dtype).contiguous() if dpooled is not None else None
        need_w = ctx.needs_input_grad[1]
        need_b = has_b and ctx.needs_input_grad[2]
        # accumulate straight into the flat fp32 gradient views when bound
        direct_w = need_w and weight.grad is not None and weight.grad.is_contiguous()
        direct_b = need_b and bias.grad is not None
        dw = weight.grad if direct_w else (torch.zeros_like(weight) if need_w else None)
        db = bias.grad if direct_b else (torch.zeros_like(bias) if need_b else None)
        dx = torch.empty((N, C, H, W), dtype=dtype, device=dev, memory_format=torch.channels_last)
        link = ctx.link
        if link is not None:
            from .hip_train import _region
            reg = _region(C, dev)
            _ext.call("mda_pool_fc_bwd_bn", dt, dlogits, dpooled, pooled, weight.detach(), dw, db,
                      dx, N, H * W, C, J, 1, link.y, link.res, link.stats, link.act, reg, link.vres)
            link.arm(dx, reg)
        else:
            _ext.call("mda_pool_fc_bwd", dt, dlogits, dpooled, pooled, weight.detach(), dw, db, dx,
                      N, H * W, C, J, 1)
        if direct_w or direct_b:
            from ..parallel.grad_reducer import notify_grad
            notify_grad(*([weight] if direct_w else []), *([bias] if direct_b else []))
        return (dx, None if direct_w else dw, None if direct_b else db)

    @staticmethod
    def _backward_dual(ctx, dpooled, dlogits):
        """DOT single-pass backward (ops.hip_train._Dual): the head kernel once
        per gradient set, into the two sets of the flat gradient and the two
        halves of one stacked dx (with one BN-sum region per set)."""
        from . import _ext
        from .hip_train import dual_full, dual_alloc, dual_ptr, _region_pair, _region_bytes
        pooled, weight, bias = ctx.saved_tensors
        N, C, H, W, J, dt, has_b = ctx.meta
        dev = pooled.device
        if dpooled is not None or dlogits is None or dlogits.dtype != pooled.dtype:
            raise RuntimeError("DOT single-pass backward: the head needs stacked logit gradients only")
        dl = dual_full(dlogits)
        if weight.grad is None or not weight.grad.is_contiguous() or (has_b and bias.grad is None):
            raise RuntimeError("DOT single-pass backward: head parameters need bound flat gradients")
        full, dx = dual_alloc((N, C, H, W), pooled.dtype, dev)
        link = ctx.link
        reg = _region_pair(C, dev) if link is not None else None
        rb = _region_bytes(C)
        for k in (0, 1):
            dw = dual_ptr(weight.grad, k)
            db = dual_ptr(bias.grad, k) if has_b else None
            dxk = full.data_ptr() + k * N * H * W * C * full.element_size()
            dlk = dl[k * N:(k + 1) * N]
            if link is not None:
                _ext.call("mda_pool_fc_bwd_bn", dt, dlk, None, pooled, weight.detach(), dw, db, dxk,
                          N, H * W, C, J, 1, link.y, link.res, link.stats, link.act,
                          reg.data_ptr() + k * rb, link.vres)
            else:
                _ext.call("mda_pool_fc_bwd", dt, dlk, None, pooled, weight.detach(), dw, db, dxk,
                          N, H * W, C, J, 1)
        if link is not None:
            link.arm(dx, reg)
        from ..parallel.grad_reducer import notify_grad
        notify_grad(weight, *([bias] if has_b else []))
        return dx, None, None


def _fc_dims(fc):
    """(in, out) of a classifier: an ``nn.Linear`` or a 1 x 1 ``nn.Conv2d`` on
    the pooled map (Tiny-ImageNet MobileNetV2's head); None otherwise."""
    if isinstance(fc, nn.Linear):
        return fc.in_features, fc.out_features
    if (isinstance(fc, nn.Conv2d) and fc.kernel_size == (1, 1) and fc.groups == 1
            and fc.stride == (1, 1) and fc.padding in ((0, 0), 0)):
        return fc.in_channels, fc.out_channels
    return None


def _pool_fc_native(x: torch.Tensor, fc, kernel) -> bool:
    if not (x.dim() == 4 and hip_enabled_for(x)):
        return False
    N, C, H, W = x.shape
    dims = _fc_dims(fc)
    if dims is None or kernel not in (None, H) or H != W or dims[0] != C \
            or fc.weight.dtype != torch.float32:
        return False
    if C > 8192 or dims[1] * C > (1 << 24) or N > 16384:
        return False
    if x.dtype == torch.bfloat16:
        return True
    return x.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")


_FP32_HEAD = {"on": False}


class fp32_head:
    """Context: classifier heads pool and project in fp32 (evaluation).

    The reference evaluates in fp32; under the bf16 step the logits would be
    bf16, whose coarse rounding creates top-k ties.  ``validate`` enables this
    so the scored logits come from an fp32 pool + fp32 GEMM of the features.
    """

    def __enter__(self):
        self._prev = _FP32_HEAD["on"]
        _FP32_HEAD["on"] = True
        return self

    def __exit__(self, *exc):
        _FP32_HEAD["on"] = self._prev
        return False


def pool_linear(x: torch.Tensor, fc: nn.Linear, kernel: int | None = None):
    """``avg = avg_pool2d(x, kernel).flatten(1); (avg, fc(avg))`` -- the CNN head.

    With a global pool (``kernel`` == spatial size, or None) on the GPU this is
    one fused HIP launch forward and one backward (:class:`_PoolFC`).
    """
    if _FP32_HEAD["on"] and not torch.is_grad_enabled():
        with torch.autocast(x.device.type, enabled=False):
            xf = x.float()
            if kernel is None:
                avg = xf.mean(dim=(2, 3))
            else:
                avg = F.avg_pool2d(xf, kernel).reshape(x.size(0), -1)
            return avg, F.linear(avg, fc.weight.float().reshape(fc.weight.shape[0], -1),
                                 fc.bias.float() if fc.bias is not None else None)
    if _pool_fc_native(x, fc, kernel):
        # (a 1 x 1 conv's [J, C, 1, 1] weight is the same memory as [J, C])
        return _PoolFC.apply(x, fc.weight, fc.bias)
    if kernel is None:
        avg = F.adaptive_avg_pool2d(x, 1).reshape(x.size(0), -1)
    else:
        avg = F.avg_pool2d(x, kernel).reshape(x.size(0), -1)
    if isinstance(fc, nn.Conv2d):
        return avg, fc(avg.reshape(avg.size(0), -1, 1, 1)).flatten(1)
    return avg, fc(avg)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """(N, C, H, W) -> (N, C), fp32-accumulated."""
    return x.float().mean(dim=(2, 3)).to(x.dtype)


class _MaxPoolNHWC(torch.autograd.Function):
    """k x k / stride / pad max pool on the HIP kernels (csrc/pool.hip):
    forward stores the argmax window offset (uint8), backward gathers."""

    @staticmethod
    def forward(ctx, x, k, s, p):
        from . import _ext
        xc = x.contiguous(memory_format=torch.channels_last)
        N, C, H, W = xc.shape
        Ho = (H + 2 * p - k) // s + 1
        Wo = (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        need = ctx.needs_input_grad[0]
        idx = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device) if need else None
        _ext.call("mda_maxpool_fwd", xc, y, idx, N, H, W, C, Ho, Wo, k, s, p)
        ctx.save_for_backward(idx)
        ctx.meta = (N, C, H, W, Ho, Wo, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _ext
        from .hip_train import _DUAL
        idx, = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        if _DUAL[0] is not None:
            return _MaxPoolNHWC._backward_dual(ctx, dy)
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=dy.device,
                         memory_format=torch.channels_last)
        _ext.call("mda_maxpool_bwd", dy, idx, dx, N, H, W, C, Ho, Wo, k, s, p)
        return dx, None, None, None

    @staticmethod
    def _backward_dual(ctx, dy):
        """DOT single-pass backward (ops.hip_train._Dual): the gather once per
        gradient set (the forward's argmax offsets serve both) into the two
        halves of one stacked dx."""
        from . import _ext
        from .hip_train import dual_full, dual_alloc
        idx, = ctx.saved_tensors
        N, C, H, W, Ho, Wo, k, s, p = ctx.meta
        if dy.dtype != torch.bfloat16 or not dy.is_contiguous(memory_format=torch.channels_last):
            raise RuntimeError("DOT single-pass backward: max-pool gradient not bf16 channels_last")
        dfull = dual_full(dy)
        full, dx = dual_alloc((N, C, H, W), torch.bfloat16, dy.device)
        for i in (0, 1):
            _ext.call("mda_maxpool_bwd", dfull[i * N:(i + 1) * N], idx, full[i * N:(i + 1) * N],
                      N, H, W, C, Ho, Wo, k, s, p)
        return dx, None, None, None


def _pair1(v):
    if isinstance(v, (tuple, list)):
        return v[0] if len(set(v)) == 1 else None
    return v


def max_pool2d(x: torch.Tensor, kernel_size, stride=None, padding=0) -> torch.Tensor:
    """``F.max_pool2d`` with a native NHWC bf16 path (square windows, no dilation)."""
    k = _pair1(kernel_size)
    s = _pair1(stride if stride is not None else kernel_size)
    p = _pair1(padding)
    if (k is not None and s is not None and p is not None and x.dim() == 4 and hip_enabled_for(x)
            and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0 and 2 * p <= k
            and x.shape[2] + 2 * p >= k and x.shape[3] + 2 * p >= k):
        return _MaxPoolNHWC.apply(x, int(k), int(s), int(p))
    return F.max_pool2d(x, kernel_size, stride, padding)


class MaxPool2d(nn.MaxPool2d):
    """Drop-in ``nn.MaxPool2d`` (same state_dict / repr) running :func:`max_pool2d`."""

    def forward(self, x):
        if self.dilation not in (1, (1, 1)) or self.ceil_mode or self.return_indices:
            return super().forward(x)
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)


_GRAD_FORKS = {"on": True}


def set_grad_forks(flag: bool) -> None:
    """A/B switch: residual-fork gradients summed in the native dgrad epilogue
    (default) or by autograd."""
    _GRAD_FORKS["on"] = bool(flag)


def grad_fork(x: torch.Tensor):
    """A :class:`ops.hip_train.GradFork` for an activation with two native
    consumers (training on the HIP path), else None."""
    if not (_GRAD_FORKS["on"] and torch.is_grad_enabled() and x.requires_grad
            and hip_enabled_for(x)):
        return None
    from . import hip_train
    return hip_train.GradFork()
