"""Training-mode conv + BatchNorm (+ residual) (+ activation) on the native kernels.

One autograd node per layer:

forward   pack weights (fp32 OIHW -> bf16 GEMM operands, one launch for all layers)
          conv          (MFMA implicit GEMM, raw output y; the epilogue also writes the
                         per-block BN statistics partials from the tile it just stored)
          bn_finalize   (channel-parallel: batch mean / rstd, scale/shift, running-stat
                         update)
          bn_apply      (z = y*scale + shift + res, out = act(z), optional preact)
backward  bn_bwd_reduce (dgamma / dbeta accumulated straight into the flat grad buffer)
          bn_bwd_apply  (dy, and dz for the residual branch)
          conv dgrad    (MFMA implicit GEMM over dy, any stride)
          conv wgrad    (MFMA with ds_read_b64_tr_b16 fragments, accumulated into
                         the fp32 OIHW grad view of the flat buffer)

Reference numerics are PyTorch's ``F.conv2d`` + ``F.batch_norm(training=True)``
(+ add + ReLU); ``tests/test_gpu_train_layers.py`` checks values and
gradients against them.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn as nn

from . import _ext
from ..parallel.grad_reducer import notify_grad

_ACT = {"none": 0, "relu": 1, "relu6": 2}


class _WS:
    """Per-stream scratch for the unfused BN reductions (partial rows +
    arrival counters)."""

    def __init__(self, device):
        self.partial = torch.zeros(2 * 2048 * 512, dtype=torch.float32, device=device)
        self.counter = torch.zeros(64, dtype=torch.int32, device=device)


_BN_FUSED = [os.environ.get("MDA_BN_FUSED", "1") != "0"]


def set_bn_fused(on: bool) -> None:
    """Fused BN (one-shot channel-sum regions: conv+stats -> apply with the
    finalize in its prologue; one-launch grid-barrier backward) vs the
    partial-rows path (A/B)."""
    _BN_FUSED[0] = bool(on)


_REG_BYTES: dict = {}


def _region_bytes(C: int) -> int:
    v = _REG_BYTES.get(C)
    if v is None:
        o = ctypes.c_int64(0)
        _ext.call("mda_bn_region_bytes", C, o)
        v = _REG_BYTES[C] = (int(o.value) + 255) // 256 * 256
    return v


class _Arena:
    """Per-device arena of one-shot BN regions (csrc/bnslot.h).

    ``bn_step_begin`` (start of every training step, inside its hipGraph)
    zeroes the part the previous steps used with ONE memset and hands regions
    out from offset 0: each training BN call of the step gets its own zeroed
    region, at the same offset in every step, so captured graphs stay valid.
    Calls outside a step, or beyond the zeroed part, get a fresh zeroed tensor.
    """

    CAP = 8 << 20

    def __init__(self, device):
        # fp32-typed so the step's memset can share one multi-tensor zeroing
        # launch with the flat fp32 gradient buffer (engine/step.py::_fwd)
        self.buf32 = torch.zeros(self.CAP // 4, dtype=torch.float32, device=device)
        self.buf = self.buf32.view(torch.uint8)
        self.err = torch.zeros(4, dtype=torch.int32, device=device)  # barrier timeouts
        self.off = 0
        self.zeroed = 0
        self.high = 64 << 10
        self.active = False


_ARENAS: dict = {}


def _arena(device) -> _Arena:
    dev = torch.device(device)
    key = dev.index or 0
    a = _ARENAS.get(key)
    if a is None:
        a = _ARENAS[key] = _Arena(dev)
    return a


def bn_step_begin(device, zero: bool = True):
    """Start a training step's arena.  ``zero=False``: the caller zeroes the
    returned fp32 view itself (e.g. in one multi-tensor launch with the
    gradients) before the step's first BN."""
    a = _arena(device)
    n = (min(a.high, a.CAP) + 255) // 256 * 256
    a.off, a.zeroed, a.active = 0, n, True
    view = a.buf32[:n // 4]
    if zero:
        view.zero_()
    return view


def bn_step_end(device) -> None:
    a = _ARENAS.get(torch.device(device).index or 0)
    if a is not None:
        a.active = False


def _region(C: int, device):
    a = _arena(device)
    need = _region_bytes(C)
    if a.active:
        start = a.off
        a.off += need
        a.high = max(a.high, a.off)  # the next step's memset covers the demand
        if a.off <= a.zeroed:
            return a.buf[start:a.off]
    return torch.zeros(need, dtype=torch.uint8, device=device)


def _region_pair(C: int, device):
    """Two adjacent zeroed regions (DOT single-pass backward: one per
    gradient set); the second starts ``_region_bytes(C)`` bytes in."""
    a = _arena(device)
    need = 2 * _region_bytes(C)
    if a.active:
        start = a.off
        a.off += need
        a.high = max(a.high, a.off)
        if a.off <= a.zeroed:
            return a.buf[start:a.off]
    return torch.zeros(need, dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------
# DOT single-pass backward.  DOT needs the task (CE) and distillation (KD)
# gradients of every parameter separately (reference engine/dot.py:15-55,
# trainer.py:425-432: two backward passes).  The backward is linear in the
# cotangent, so both passes are run as ONE over two stacked cotangents: every
# native backward of the student receives a gradient that is the first half
# of a [2N, ...] buffer (set 0 = KD, set 1 = CE), processes both halves in the
# same launches (dgrad over 2N images, BN backward with gridDim.y = 2 and one
# region per set, wgrad into both gradient sets of the flat buffer) and hands
# on the first half of a new stacked buffer.  The autograd engine only ever
# sees the set-0 views, so its shape checks hold; any op outside the native
# kernels that would touch such a gradient (a PyTorch add, a cast) breaks the
# pairing, which :func:`dual_full` detects and refuses loudly.
class _Dual:
    __slots__ = ("gstride", "halves")

    def __init__(self, gstride):
        self.gstride = int(gstride)   # set-1 gradient = set-0 view + gstride floats
        # base address -> (the set-0 half handed to autograd, its _version): a
        # gradient is accepted only if it IS that tensor, unmodified -- an
        # in-place accumulation by autograd (InputBuffer add) bumps the version
        self.halves = {}


_DUAL = [None]


def set_dual(gstride) -> None:
    """Arm (``gstride`` = float offset from the bound gradient set to the other
    set of the flat buffer) or disarm (None) the single-pass DOT backward."""
    _DUAL[0] = _Dual(gstride) if gstride is not None else None


def dual_active() -> bool:
    return _DUAL[0] is not None


def dual_alloc(shape, dtype, device, channels_last=True):
    """-> (stacked [2N, ...] buffer, its set-0 half)."""
    fmt = torch.channels_last if (channels_last and len(shape) == 4) else torch.contiguous_format
    full = torch.empty((2 * shape[0],) + tuple(shape[1:]), dtype=dtype, device=device,
                       memory_format=fmt)
    half = full[:shape[0]]
    _DUAL[0].halves[full.data_ptr()] = (half, half._version)
    return full, half


def dual_seal(half) -> None:
    """Re-record ``half``'s version after a PyTorch op wrote its stacked buffer
    (``torch.add(..., out=full)``): the write is ours, not autograd's."""
    D = _DUAL[0]
    if D is not None and half.data_ptr() in D.halves:
        D.halves[half.data_ptr()] = (half, half._version)


def dual_full(g):
    """The stacked [2N, ...] buffer whose first half is the gradient ``g``."""
    if g is None:
        return None
    D = _DUAL[0]
    rec = D.halves.get(g.data_ptr()) if D is not None else None
    if (rec is None or rec[0] is not g or g._version != rec[1] or g.storage_offset() != 0):
        raise RuntimeError(
            "DOT single-pass backward: a gradient reached a native layer without its stacked "
            "second set (a non-native op in the student's backward?); set "
            "RUNTIME.DOT_SINGLE_PASS=False for this model")
    return g.as_strided((2 * g.shape[0],) + tuple(g.shape[1:]), g.stride())


def dual_ptr(t, k: int):
    """Device address of set ``k`` of a flat-gradient view ``t`` (set 0 = ``t``)."""
    return t.data_ptr() + (4 * _DUAL[0].gstride if k else 0)


def _err_word(device):
    return _arena(device).err


def slot_errors() -> int:
    """Number of devices on which a fused-BN grid barrier timed out (must be 0)."""
    return sum(int(a.err.max().item() != 0) for a in _ARENAS.values())


_WSS: dict = {}
_WS_TAG = [None]


def set_ws_tag(tag) -> None:
    """Give the BN scratch of the code that follows its own buffers: a graph
    captured under a tag may be replayed concurrently with one captured on the
    same stream without it (DOT's task and KD backwards, engine/step.py)."""
    _WS_TAG[0] = tag


def _ws(device):
    # one scratch buffer PER STREAM (and tag): the teacher's train-mode BN (OFD)
    # runs on the teacher stream concurrently with the student's BN kernels,
    # and a shared partials buffer raced under hipGraph replay (NaN OFD losses)
    dev = torch.device(device)
    key = (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream, _WS_TAG[0])
    w = _WSS.get(key)
    if w is None:
        w = _WSS[key] = _WS(device)
    return w


_WG_DEFER = [None]  # rows of deferred split reductions while armed (a list), else None
_WG_KEEP: list = []  # their partial buffers, alive until the flush has been queued


def set_wgrad_defer(on: bool) -> None:
    """Arm / disarm deferred weight-gradient reductions: while armed, each
    native conv backward queues only its wgrad GEMM, and
    :func:`flush_wgrad_reduces` reduces every layer's split partials into the
    flat gradient in one multi-layer launch (``mda_wgrad_reduce_multi``)
    instead of one reduce kernel per layer on the backward's critical path."""
    _WG_DEFER[0] = [] if on else None
    _WG_KEEP.clear()
    _WG_PEND[0] = None


# A deferred weight-gradient GEMM waiting to ride in the launch of the next
# BN-backward apply on the same stream (mda_conv_wgrad_nored_bn): the GEMM
# reads dy and x of its conv, the apply the dgrad output below it, so the two
# are independent and one launch fills the CUs either leaves idle.  At most
# one is parked; it holds its operands (the allocator cannot reuse them) and
# is launched on its own by the next park, the next flush, or when the apply
# is not served.  Only while the reductions are deferred (captured backward).
_WG_PEND = [None]   # (stream, wgrad args, keep-alive tensors)
_WG_FUSE_ON = [os.environ.get("MDA_WGRAD_BN_FUSE", "1") != "0"]
_WG_FUSE_COUNT = [0]  # fused launches issued (tests)


def set_wgrad_bn_fuse(on: bool) -> None:
    """Weight-gradient GEMM + next BN-backward apply in one launch on / off (A/B)."""
    _WG_FUSE_ON[0] = bool(on)


def _launch_pending_wgrad() -> None:
    pend, _WG_PEND[0] = _WG_PEND[0], None
    if pend is None:
        return
    stream, args, _ = pend
    with torch.cuda.stream(stream):
        _ext.call("mda_conv_wgrad_nored", *args)


def flush_wgrad_reduces() -> None:
    _launch_pending_wgrad()
    rows = _WG_DEFER[0]
    if rows:
        t = torch.tensor(rows, dtype=torch.int64)
        _ext.call("mda_wgrad_reduce_multi", t, len(rows))
        rows.clear()
    _WG_KEEP.clear()


def _conv_wgrad(x, dy, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kp, sp, direct,
                cin_keep, groups, nsets=1, gstride=0):
    """Weight gradient of one conv into ``target`` (accumulated when ``direct``).
    ``nsets`` = 2 (DOT single-pass backward): dy holds two stacked cotangents,
    set 1's gradient goes ``gstride`` floats past ``target`` -- one launch."""
    part = torch.empty(nsets * sp * Cout * Kp, dtype=torch.float32, device=x.device)
    if direct and _WG_DEFER[0] is not None:
        args = (x, dy, part, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kp, sp, 1.0, 1,
                cin_keep, groups, nsets)
        _launch_pending_wgrad()
        if nsets == 1 and _WG_FUSE_ON[0] and _DUAL[0] is None:
            # park it: the next BN-backward apply on this stream launches it too
            _WG_PEND[0] = (torch.cuda.current_stream(), args, (x, dy))
        else:
            _ext.call("mda_conv_wgrad_nored", *args)
        for k in range(nsets):
            _WG_DEFER[0].append([part.data_ptr() + 4 * k * sp * Cout * Kp,
                                 target.data_ptr() + 4 * k * gstride, sp, Cout, Cin, KH, KW, Kp, 1,
                                 cin_keep, groups])
        _WG_KEEP.append(part)
        return
    _ext.call("mda_conv_wgrad", x, dy, part, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
              pad, Kp, sp, 1.0, 1 if direct else 0, cin_keep, groups, nsets, gstride)


def _bn_bwd_reduce(dout, dpre, y, res, stats, M, C, act, ws, sums, dg, db):
    """dbeta / dgamma sums of the BN backward: per-block partials combined by a
    separate channel-parallel finalize launch (the in-kernel last-arriver
    combine, ``mda_bn_bwd_reduce``, measured slower: profiles/r2_misc_ab.md)."""
    _ext.call("mda_bn_bwd_reduce2", dout, dpre, y, res, stats[2], stats[3], stats[0], stats[1],
              M, C, act, ws.partial, sums, dg, db)


class BnLink:
    """A training BN layer's output, as seen by the conv that consumes it.

    The consumer's dgrad produces exactly this layer's output gradient, so its
    epilogue can also add the layer's backward channel sums (sum dz,
    sum dz*xhat) into a fresh region (``mda_conv_dgrad_bnsum``, :meth:`arm`);
    the layer's backward then runs ONE streaming pass on them
    (``mda_bn_bwd_apply_reg``) instead of a reduction + grid barrier + apply.
    The sums are used only if the gradient the layer receives IS that dgrad
    output, unmodified (:meth:`take`): if autograd summed another gradient into
    it (a feature loss on the activation, a second consumer on a non-native
    path) the tensor differs and the layer falls back to the full backward.
    The link keeps a reference to the armed tensor, so autograd never
    accumulates into it in place.
    """

    __slots__ = ("y", "res", "stats", "act", "M", "C", "dout", "ver", "region", "vres")

    def __init__(self, y, res, stats, act, M, C, vres=None):
        self.y, self.res, self.stats, self.act, self.M, self.C = y, res, stats, act, M, C
        self.vres = vres if res is not None else None  # res is a virtual residual (VirtualBN)
        self.dout = self.region = None
        self.ver = -1

    def arm(self, dout, region) -> None:
        self.dout, self.ver, self.region = dout, dout._version, region

    def take(self, dout):
        """The dgrad-epilogue sums' region when ``dout`` IS the armed tensor,
        unmodified; else None."""
        d, r = self.dout, self.region
        self.dout = self.region = None
        if d is not None and d is dout and dout._version == self.ver:
            _BNB_COUNT[0] += 1
            return r
        if d is not None:
            _BNB_COUNT[1] += 1
        return None


_BNB_COUNT = [0, 0]  # BN backwards on dgrad-epilogue sums / armed links that fell back
_LAST_VBN = [None]
_BNB_ON = [os.environ.get("MDA_BN_DGRAD_SUMS", "1") != "0"]
_LAST_LINK = [None]


def set_bn_dgrad_sums(on: bool) -> None:
    """BN-backward sums in the consumer dgrad's epilogue (BnLink) on / off (A/B)."""
    _BNB_ON[0] = bool(on)


def bn_dgrad_sums_count(reset: bool = False):
    """(BN backwards that used dgrad-epilogue sums, armed links that fell back)."""
    v = tuple(_BNB_COUNT)
    if reset:
        _BNB_COUNT[0] = _BNB_COUNT[1] = 0
    return v


def _bn_bwd(dout, dpre, y, res, stats, gamma, beta, M, C, act, need_res, direct_gb, link=None,
            res_link=None, vres=None):
    """BN (+ residual) (+ activation) backward -> (dy, dres or None, sums or
    None).  Fused: ONE grid-barrier launch (mda_bn_bwd_fused); else the
    partial-rows reduce + finalize + apply (3 launches).  dgamma / dbeta are
    accumulated into the parameters' flat-gradient views when ``direct_gb``,
    else returned through ``sums`` ([sum dz | sum dz*xhat])."""
    dev = y.device
    ws = _ws(dev)
    dg = gamma.grad if direct_gb else None
    db = beta.grad if direct_gb else None
    dy = torch.empty_like(y)
    dres = torch.empty_like(y) if need_res else None
    reg = link.take(dout) if link is not None else None
    # the residual's producer is a training BN without activation (a projection
    # shortcut): dres IS its output gradient, so this pass adds its sums too
    rl = res_link if (need_res and res_link is not None and 256 % (C // 8) == 0) else None
    rreg = _region(C, dev) if rl is not None else None
    ry, rst = (rl.y, rl.stats) if rl is not None else (None, None)
    if reg is not None and dpre is None:
        sums = None if direct_gb else torch.empty(2, C, dtype=torch.float32, device=dev)
        pend = _WG_PEND[0]
        rc = _ext.NOT_SERVED
        if pend is not None and pend[0] == torch.cuda.current_stream():
            # the parked weight-gradient GEMM and this apply in one launch
            a = pend[1]
            rc = _ext.call("mda_conv_wgrad_nored_bn", *a[:17], *a[19:21], dout, y, res, stats, M, C,
                           act, reg, dy, dres, dg, db, sums, ry, rst, rreg, vres,
                           ok=(0, _ext.NOT_SERVED))
            if rc == 0:
                _WG_PEND[0] = None
                _WG_FUSE_COUNT[0] += 1
        if rc != 0:
            _ext.call("mda_bn_bwd_apply_reg", dout, None, y, res, stats, M, C, act, reg, dy, dres,
                      dg, db, sums, ry, rst, rreg, vres, 1, 0, 0, 0)
        if rl is not None:
            rl.arm(dres, rreg)
        return dy, dres, sums
    if _BN_FUSED[0]:
        sums = None if direct_gb else torch.empty(2, C, dtype=torch.float32, device=dev)
        _ext.call("mda_bn_bwd_fused", dout, None, dpre, y, res, stats, M, C, act, _region(C, dev),
                  _err_word(dev), dy, dres, dg, db, sums, ry, rst, rreg, vres, 1, 0, 0, 0)
        if rl is not None:
            rl.arm(dres, rreg)
        return dy, dres, sums
    if vres is not None:
        raise RuntimeError("virtual residuals need the fused BN kernels (MDA_BN_FUSED=1)")
    sums = torch.empty(2, C, dtype=torch.float32, device=dev)
    _bn_bwd_reduce(dout, dpre, y, res, stats, M, C, act, ws, sums, dg, db)
    _ext.call("mda_bn_bwd_apply", dout, dpre, y, res, stats[2], stats[3], stats[0], stats[1],
              sums, dy, dres, M, C, act)
    return dy, dres, sums


_WG_PLANS: dict = {}


def _wgrad_splits(M, Cout, Cin, KH, KW, Kp, H, W, stride, pad):
    key = (M, Cout, Cin, KH, KW, Kp, H, W, stride, pad)
    v = _WG_PLANS.get(key)
    if v is None:
        s = ctypes.c_int64(0)
        _ext.call("mda_wgrad_plan", M, Cout, Cin, KH, KW, Kp, H, W, stride, pad, s)
        v = _WG_PLANS[key] = s.value
    return v


class PackCache:
    """Packed bf16 GEMM operands of every student conv, refreshed by ONE launch per step.

    The first (eager) forward of a layer packs it on its own and registers
    persistent ``wf``/``wt`` buffers; from then on :meth:`pack_all` (called by
    the training step before the forward, and captured into its hipGraph)
    repacks every registered layer in a single ``mda_pack_conv_weights_multi``
    launch and *arms* the cache, so the layers' forwards reuse the buffers
    instead of launching one pack kernel each.  :meth:`disarm` after the
    forward keeps any later, out-of-step call from seeing stale weights.
    """

    def __init__(self):
        self.entries: dict = {}
        self.armed = False
        self._table = None
        self._dirty = False
        self._total = 0
        self._extra_key = None  # (zero fills, image) the table was built with
        self._img_pad = None
        # the table / padded image a captured graph points at: an eager step
        # after the capture (a partial batch) may rebuild the table, and the
        # graph's copies must outlive that
        self._graph_refs = None

    def lookup_pad(self, weight):
        """The channel-padded stem operand packed for this step, or None."""
        if not self.armed:
            return None
        e = self.entries.get(id(weight))
        if e is None or e["weight"] is not weight or e.get("kind") != "pad":
            return None
        return e

    def register_pad(self, weight, wf, Cout, C, Cp, KH, KW, Kp):
        """A stem whose 3-channel input runs padded to ``Cp`` (``needs_channel_pad``)."""
        if torch.cuda.is_current_stream_capturing():
            return
        self.entries[id(weight)] = dict(weight=weight, wf=wf, wt=None, kind="pad",
                                        meta=(Cout, -2, KH, KW, Kp, C | (Cp << 16)))
        self._dirty = True

    def lookup(self, weight, need_dx):
        if not self.armed:
            return None
        e = self.entries.get(id(weight))
        if (e is None or e["weight"] is not weight or (need_dx and e["wt"] is None)
                or e.get("kind") == "pad"):
            return None
        return e

    def register(self, weight, wf, wt, Cout, Cin, KH, KW, Kp, KpT, groups=1):
        """``groups`` > 1: a grouped conv's compact operands (Cin = channels per
        group), packed as ``groups`` dense sub-layers: group g's OIHW rows are
        contiguous, and so are its rows of wf ([Cout][Kp]) and of wt
        ([Cin_total][KpT], k = tap * Cout/G + co)."""
        if torch.cuda.is_current_stream_capturing():
            return
        self.entries[id(weight)] = dict(weight=weight, wf=wf, wt=wt, meta=(Cout, Cin, KH, KW, Kp, KpT),
                                        groups=groups)
        self._dirty = True

    def register_dw(self, weight, wp):
        """Depthwise weight: fp32 tap-major [9, C] operand, refreshed by the same launch."""
        if torch.cuda.is_current_stream_capturing():
            return
        C = weight.shape[0]
        self.entries[id(weight)] = dict(weight=weight, wf=wp, wt=None, meta=(C, -1, 3, 3, 0, 0))
        self._dirty = True

    def _build(self, device, zero=(), image=None):
        rows, start = [], 0
        for e in self.entries.values():
            Cout, Cin, KH, KW, Kp, KpT = e["meta"]
            if Cin == -2:  # channel-padded stem: 256 packed elements per tile
                rows.append([e["weight"].data_ptr(), e["wf"].data_ptr(), 0, Cout, -2, KH, KW, Kp, KpT,
                             start])
                start += (Cout * Kp + 255) // 256
                continue
            if Cin < 0:  # depthwise row: 256 packed elements per tile
                n = (9 * Cout + 255) // 256
            else:
                t = ctypes.c_int64(0)
                _ext.call("mda_pack_tiles", Cout, Cin, KH, KW, t)
                n = t.value  # tiles of this layer (padding stays zero from registration)
            w = e["weight"]
            G = e.get("groups", 1)
            if G > 1:
                cog = Cout // G
                t = ctypes.c_int64(0)
                _ext.call("mda_pack_tiles", cog, Cin, KH, KW, t)
                for g in range(G):
                    rows.append([w.data_ptr() + 4 * g * cog * Cin * KH * KW,
                                 e["wf"].data_ptr() + 2 * g * cog * Kp,
                                 e["wt"].data_ptr() + 2 * g * Cin * KpT if e["wt"] is not None else 0,
                                 cog, Cin, KH, KW, Kp, KpT, start])
                    start += t.value
                continue
            rows.append([w.data_ptr(), e["wf"].data_ptr(), e["wt"].data_ptr() if e["wt"] is not None else 0,
                         Cout, Cin, KH, KW, Kp, KpT, start])
            start += n
        for t in zero:  # the step's zero fills ride in the same launch
            nb = t.numel() * t.element_size()
            rows.append([t.data_ptr(), nb, 0, 0, -3, 1, 1, 0, 0, start])
            start += (nb + 16383) // 16384
        if image is not None:
            N, C, H, W = image.shape
            if self._img_pad is None or tuple(self._img_pad.shape) != (N, 8, H, W):
                self._img_pad = torch.empty((N, 8, H, W), dtype=torch.bfloat16, device=device,
                                            memory_format=torch.channels_last)
            M = N * H * W
            rows.append([image.data_ptr(), self._img_pad.data_ptr(),
                         0 if image.dtype == torch.float32 else 1, M, -4, C, 1, 0, 0, start])
            start += (M + 255) // 256
        self._table = torch.tensor(rows, dtype=torch.int64).to(device)
        self._total = start
        self._khkw = max(r[5] * r[6] for r in rows if r[4] != -2)
        self._ptrs = [e["weight"].data_ptr() for e in self.entries.values()]
        self._extra_key = self._key(zero, image)
        self._dirty = False

    @staticmethod
    def _key(zero, image):
        return (tuple((t.data_ptr(), t.numel() * t.element_size()) for t in zero),
                None if image is None else (image.data_ptr(), tuple(image.shape), image.dtype))

    @staticmethod
    def _image_ok(image) -> bool:
        return (image is not None and image.dim() == 4 and needs_channel_pad(image.shape[1])
                and image.dtype in (torch.float32, torch.bfloat16)
                and image.is_contiguous(memory_format=torch.channels_last))

    def pack_all(self, device, zero=(), image=None) -> bool:
        """Repack every registered layer in one launch (and arm the cache).
        ``zero``: tensors to zero-fill in the same launch (4-byte multiples);
        ``image``: a 3-channel NHWC image whose 8-channel padded copy the stem
        then reads (:func:`pad_channels8`), built in the same launch -- only
        for a stable buffer (the captured step's static input).  Returns False
        having launched nothing (the caller zeroes ``zero`` itself)."""
        image = image if self._image_ok(image) else None
        nrows = sum(e.get("groups", 1) for e in self.entries.values()) + len(zero) + (image is not None)
        if not self.entries or nrows > 256 or any(
                e["meta"][2] * e["meta"][3] > 49 for e in self.entries.values()):
            return False
        if any(t.numel() * t.element_size() % 4 or t.data_ptr() % 16 or not t.is_contiguous()
               for t in zero):
            return False
        capturing = torch.cuda.is_current_stream_capturing()
        stale = self._table is None or self._dirty or any(
            e["weight"].data_ptr() != p for e, p in zip(self.entries.values(), self._ptrs)
        ) or self._extra_key != self._key(zero, image)
        if stale:
            if capturing:
                return False
            self._build(device, zero, image)
        _ext.call("mda_pack_conv_weights_multi", self._table, self._table.shape[0], self._total,
                  self._khkw)
        if capturing:
            self._graph_refs = (self._table, self._img_pad)
        self.armed = True
        _PREPAD[0] = ((image, image._version, self._img_pad, torch.cuda.current_stream(device).cuda_stream)
                      if image is not None else None)
        return True

    def disarm(self):
        self.armed = False
        _PREPAD[0] = None


_PREPAD = [None]  # (image, version, its 8-channel copy, stream) built by the armed PackCache


_ACTIVE = [None]  # the PackCache of the training step currently running its forward


def set_active_packs(cache) -> None:
    _ACTIVE[0] = cache


def _cl_bf16(t):
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


def needs_channel_pad(cin: int) -> bool:
    """3-channel image convs run on the 16-byte vector loaders with the input
    zero-padded to 8 channels (``mda_pad_channels``)."""
    return cin < 8 and cin % 8 != 0


def pad_channels8(x):
    """NCHW-logical (any layout) fp32/bf16 image -> bf16 channels_last with 8
    channels (zeros beyond the real ones), one launch.  Cached per tensor
    version and stream, so a second consumer on the same stream (e.g. two
    stems) reuses it."""
    pp = _PREPAD[0]
    # built by this step's multi-pack launch (PackCache.pack_all) -- on that
    # launch's stream only: a teacher on its own stream pads for itself
    if (pp is not None and pp[0] is x and pp[1] == x._version
            and pp[3] == torch.cuda.current_stream(x.device).cuda_stream):
        return pp[2]
    key = (x._version, torch.cuda.current_stream(x.device).cuda_stream)
    # never across a graph capture: a hit would leave the pad kernel out of the
    # graph, whose replays then read the padded copy of the capture-time image
    capturing = torch.cuda.is_current_stream_capturing()
    cache = getattr(x, "_mda_pad8", None)
    if cache is not None and cache[0] == key and not capturing:
        return cache[1]
    xc = x.contiguous(memory_format=torch.channels_last)
    if xc.dtype not in (torch.float32, torch.bfloat16):
        xc = xc.float()
    N, C, H, W = xc.shape
    y = torch.empty((N, 8, H, W), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    _ext.call("mda_pad_channels", 0 if xc.dtype == torch.float32 else 1, xc, y, N * H * W, C, 8)
    try:
        if capturing:
            x.__dict__.pop("_mda_pad8", None)
        else:
            x._mda_pad8 = (key, y)
    except Exception:  # noqa: BLE001 -- caching is optional
        pass
    return y


_GROUPED_NATIVE = [os.environ.get("MDA_GROUPED_NATIVE", "0") == "1"]


def set_grouped_native(on: bool) -> None:
    _GROUPED_NATIVE[0] = bool(on)


_GROUPED_COMPACT = [os.environ.get("MDA_GROUPED_COMPACT", "1") != "0"]


def set_grouped_compact(on: bool) -> None:
    """Grouped convs on compact per-group operands (default) vs the dense
    block-diagonal GEMM (A/B, and the path for unaligned groups)."""
    _GROUPED_COMPACT[0] = bool(on)


_DET = {"on": False, "saved": None}


def set_deterministic(on: bool) -> None:
    """Deterministic mode (``EXPERIMENT.DETERMINISTIC``): every
    reduction of the native training path in a fixed order, so two runs of
    the same step are bitwise equal.  The fast path sums BN batch / backward
    statistics with fp64 atomics into one-shot regions (csrc/bnslot.h: in the
    conv and depthwise epilogues, the consumer dgrad's BN-sum epilogue, the
    pool + FC head) whose order varies run to run; here BN runs on per-block
    partial rows and a fixed-order finalize launch instead (the
    ``MDA_BN_FUSED=0`` kernels), and the fusions that exist only on the
    regions (VirtualBN, BnLink sums) are off.  Everything else is fixed-order in both modes (split-K
    combines, weight-gradient partial reduces, losses, optimizer, VID).
    Turning it off restores the switches as they were."""
    on = bool(on)
    if on == _DET["on"]:
        return
    if on:
        _DET["saved"] = (_BN_FUSED[0], _BNB_ON[0], _VRES_ON[0])
        _BN_FUSED[0] = _BNB_ON[0] = _VRES_ON[0] = False
    else:
        (_BN_FUSED[0], _BNB_ON[0], _VRES_ON[0]) = _DET["saved"]
    _DET["on"] = on


def deterministic() -> bool:
    return _DET["on"]


def train_supported(x, conv, bn) -> bool:
    if not (x.is_cuda and x.dim() == 4 and isinstance(conv, nn.Conv2d)):
        return False
    if bn is None or not bn.training or not bn.track_running_stats or bn.momentum is None:
        return False
    if conv.dilation != (1, 1) or conv.padding_mode != "zeros":
        return False
    # a conv bias in front of a training BN only shifts the batch mean (BN
    # removes it; its gradient sum_m dy is exactly 0): the conv runs without it
    # and the running mean takes the shift (_ConvBNActTrain)
    # (depthwise too: Tiny-ImageNet MobileNetV2's depthwise convs carry biases)
    if conv.bias is not None and ((conv.groups != 1 and not is_depthwise(conv))
                                  or conv.bias.dtype != torch.float32):
        return False
    if conv.groups != 1:
        if is_depthwise(conv):
            return dw_train_supported(x, conv, bn)
        # grouped (ShuffleNetV1): one dense GEMM on the block-diagonal weight.
        # Opt-in (MDA_GROUPED_NATIVE=1): G x the MFMA work plus a per-call pack
        # measured slower than MIOpen's grouped kernels on ShuffleV1 (5.48 vs
        # 5.34 ms/step, profiles/r2_misc_ab.md); the GPU test runs it either way.
        cig, cog = conv.in_channels // conv.groups, conv.out_channels // conv.groups
        if conv.in_channels % 8 or conv.out_channels % 8:
            return False
        # compact grouped GEMM when every group is 16-byte aligned; the
        # block-diagonal dense fallback only on request
        if (cig % 8 or cog % 8) and not _GROUPED_NATIVE[0]:
            return False
    if conv.stride[0] != conv.stride[1] or not isinstance(conv.padding, tuple) or conv.padding[0] != conv.padding[1]:
        return False
    if conv.kernel_size[0] != conv.kernel_size[1]:
        return False
    if conv.out_channels % 8 or (conv.in_channels % 8 and x.requires_grad):
        return False
    if bn.weight is None or bn.bias is None:
        return False
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    return torch.is_grad_enabled()


def is_depthwise(conv) -> bool:
    return (conv.groups > 1 and conv.groups == conv.in_channels == conv.out_channels)


def dw_supported_geometry(conv) -> bool:
    """3x3 depthwise, stride 1/2, square padding (csrc/dwconv.hip)."""
    return (is_depthwise(conv) and conv.kernel_size == (3, 3) and conv.stride[0] == conv.stride[1]
            and conv.stride[0] in (1, 2) and isinstance(conv.padding, tuple)
            and conv.padding[0] == conv.padding[1] and conv.dilation == (1, 1)
            and conv.padding_mode == "zeros" and conv.out_channels <= 2048)


def dw_train_supported(x, conv, bn) -> bool:
    if not dw_supported_geometry(conv) or bn is None or bn.weight is None or bn.bias is None:
        return False
    if conv.out_channels % 8:  # BN kernels are 8-channel vectorised
        return False
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    return torch.is_grad_enabled()


def dw_pack(weight, scale=None):
    """fp32 [C, 1, 3, 3] -> fp32 tap-major [9, C] (optionally scaled per channel)."""
    C = weight.shape[0]
    out = torch.empty(9, C, dtype=torch.float32, device=weight.device)
    _ext.call("mda_dw_pack", weight.detach().float().contiguous(), scale, out, C, 9)
    return out


def _dw_wgrad_blocks(N, H, W, C, Ho, Wo, stride, pad=1):
    key = ("dw", N, H, W, C, Ho, Wo, stride, pad)
    v = _WG_PLANS.get(key)
    if v is None:
        b = ctypes.c_int64(0)
        _ext.call("mda_dw_wgrad_blocks2", N, H, W, C, Ho, Wo, stride, pad, b)
        v = _WG_PLANS[key] = b.value
    return v


class GradFork:
    """Two consumers of one activation (a residual fork: conv1 and the
    shortcut conv, or conv1 and the identity residual) whose input gradients
    are summed INSIDE the native backward instead of by an autograd add.

    Both consumers register in their forward (:meth:`join`); in the backward
    the first one to run parks its gradient (and an event on its stream) and
    returns None for the shared input; the second adds the parked gradient in
    its dgrad's residual epilogue (``mda_conv_dgrad_res``) -- or, if it has no
    dgrad, with one add -- and returns the sum.  A fork whose second consumer
    took a non-native path (``members < 2``) is inert: both return their own
    gradient and autograd adds them as usual.
    """

    def __init__(self):
        self.members = 0
        self.pending = None
        self.event = None

    def join(self):
        self.members += 1
        return self

    @property
    def armed(self) -> bool:
        return self.members == 2

    def park(self, g) -> bool:
        """First arrival: keep ``g`` (a gradient, or a :class:`_DeferredDgrad`)
        and return True (caller returns None)."""
        if not self.armed or self.pending is not None:
            return False
        self.pending = g
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(g.device))
        return True

    def take(self):
        """Second arrival: the parked gradient (ordered on the current stream) --
        a tensor, or a :class:`_DeferredDgrad` -- or None."""
        if not self.armed or self.pending is None:
            return None
        g, self.pending = self.pending, None
        cur = torch.cuda.current_stream(g.device)
        cur.wait_event(self.event)
        for t in (g.tensors() if isinstance(g, _DeferredDgrad) else (g,)):
            t.record_stream(cur)
        self.event = None
        return g


class _DeferredDgrad:
    """A 1 x 1 / stride-s / pad-0 conv's input gradient, not computed: its
    output gradient ``dy`` and dgrad operand ``wt`` parked on the residual fork
    for the other consumer's dgrad to fold in (``mda_conv_dgrad_bnsum2``)."""

    __slots__ = ("dy", "wt", "cin2", "kp2", "stride", "device")

    def __init__(self, dy, wt, cin2, kp2, stride):
        self.dy, self.wt, self.cin2, self.kp2, self.stride = dy, wt, cin2, kp2, stride
        self.device = dy.device

    def tensors(self):
        return (self.dy, self.wt)

    def materialize(self, x_shape):
        """The input gradient itself (the fold was not served)."""
        from .hip_layers import conv_plan
        N, Cin, H, W = x_shape
        dx = torch.empty(x_shape, dtype=torch.bfloat16, device=self.device,
                         memory_format=torch.channels_last)
        Ho, Wo = self.dy.shape[2], self.dy.shape[3]
        tile, splits = conv_plan(N * H * W, Cin, self.kp2)
        part = (torch.empty(splits * N * H * W * Cin, dtype=torch.float32, device=self.device)
                if splits > 1 else None)
        _ext.call("mda_conv_dgrad", self.dy, self.wt, dx, part, N, H, W, Cin, Ho, Wo, self.cin2,
                  1, 1, self.stride, 0, self.kp2, tile, splits)
        return dx


_MERGE_ON = [os.environ.get("MDA_DGRAD_MERGE", "1") != "0"]
_MERGE_COUNT = [0]  # folded dgrads launched (tests)


def set_dgrad_merge(on: bool) -> None:
    """A projection shortcut's input gradient folded into conv1's dgrad on / off (A/B)."""
    _MERGE_ON[0] = bool(on)


def _fork_sum(fork, g):
    """Autograd-visible gradient of a forked input for a consumer without a
    dgrad of its own (the identity residual): park it, or add the parked one."""
    if fork is None or g is None:
        return g
    if fork.park(g):
        return None
    other = fork.take()
    if other is None:
        return g
    if isinstance(other, _DeferredDgrad):
        # a parked projection-shortcut dgrad whose fold partner has no dgrad
        # of its own: compute it here
        if _DUAL[0] is not None:
            raise RuntimeError("a deferred shortcut dgrad reached the dual backward")
        other = other.materialize(tuple(g.shape))
    if _DUAL[0] is not None:
        gf, of = dual_full(g), dual_full(other)
        full, half = dual_alloc(g.shape, g.dtype, g.device)
        torch.add(gf, of, out=full)
        dual_seal(half)
        return half
    return g + other


class VirtualBN:
    """A training conv + BN whose apply pass was folded into its consumer's.

    A projection shortcut's BN has no activation and its only consumer is the
    block's last apply (``act(bn2(y2) + bn_sc(y_sc))``): the shortcut conv
    only accumulates its batch sums (``region``), its autograd output is the
    RAW conv output ``y_sc``, and the consumer's ``mda_bn_apply_fin_vr``
    finalizes both BNs and adds ``y_sc * scale_sc + shift_sc`` -- one apply
    launch per downsampling block instead of two.  Every later pass that
    recomputes the block's pre-activation (the BN backward, the consumer
    dgrad's BN-sum epilogue, the pool+FC head) gets the shortcut's [4][C]
    stats as ``vres`` and applies the same affine to the raw residual.
    """

    __slots__ = ("reg", "gamma", "beta", "bn", "stats")

    def __init__(self, reg, gamma, beta, bn, stats):
        self.reg, self.gamma, self.beta, self.bn, self.stats = reg, gamma, beta, bn, stats


_VRES_ON = [os.environ.get("MDA_VIRTUAL_RES", "1") != "0"]


def set_virtual_residual(on: bool) -> None:
    """Projection-shortcut BN applied inside the block's last apply (VirtualBN) on / off (A/B)."""
    _VRES_ON[0] = bool(on)


def can_defer_residual(h, conv, bn) -> bool:
    """The block's residual consumer (conv ``conv`` + ``bn`` on input ``h``)
    runs on the native training kernels, so a projection shortcut may hand it
    a :class:`VirtualBN` output."""
    return (_VRES_ON[0] and _BN_FUSED[0] and h is not None and h.is_cuda and conv.groups == 1
            and train_supported(h, conv, bn))


# A residual block's conv1 BN apply rides in the launch of its projection
# shortcut's conv (csrc/conv1x1.hip mda_conv1x1_bnacc_apply): neither reads
# the other's output, and back to back each ran on half the GPU.  The block
# arms it (arm_apply_ride) with its input; conv1's forward then PARKS its
# plain BN apply instead of launching it, the shortcut conv on the same input
# launches both, and finish_apply_ride launches a parked apply that found no
# rider (a shortcut that is not a streaming-kernel shape).  Nothing reads
# conv1's BN output before the shortcut: conv2 runs after it.
_RIDE = {"x": None, "apply": None}
_RIDE_ON = [os.environ.get("MDA_APPLY_RIDE", "1") != "0"]
_RIDE_COUNT = [0]  # fused launches issued (tests)


def set_apply_ride(on: bool) -> None:
    """conv1's BN apply riding in the projection shortcut's launch on / off (A/B)."""
    _RIDE_ON[0] = bool(on)


def arm_apply_ride(x) -> None:
    _flush_apply_ride()
    _RIDE["x"] = x if (_RIDE_ON[0] and _BN_FUSED[0] and x is not None and x.is_cuda
                       and torch.is_grad_enabled()) else None


def _flush_apply_ride() -> None:
    pend, _RIDE["apply"] = _RIDE["apply"], None
    if pend is not None:
        stream, args, _ = pend
        with torch.cuda.stream(stream):
            _ext.call("mda_bn_apply_fin", *args)


def finish_apply_ride() -> None:
    _RIDE["x"] = None
    _flush_apply_ride()


class _ConvBNActTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, gamma, beta, residual, meta, bn, want_preact, forks=(None, None),
                cbias=None, defer=False, private=False):
        # an unused output (the pre-activation) must not be materialised as a
        # zero gradient + layout copy: the kernels take null dout / dpre
        ctx.set_materialize_grads(False)
        stride, pad, act = meta[:3]
        if len(meta) > 3 and meta[3] == "dw":
            ctx.forks = (None, None)
            ctx.cbias = cbias is not None
            ctx.cbias_t = cbias
            res = _dw_forward(ctx, x, weight, gamma, beta, residual, stride, pad, act, bn,
                              want_preact)
            if cbias is not None:
                # BN(y + b) == BN(y) in training; the running mean (updated by the
                # BN kernel above) tracks mean(y) + b (same algebra as the dense path)
                bn.running_mean.add_(cbias.detach(), alpha=float(bn.momentum))
            return res
        ctx.kind = "dense"
        ctx.forks = tuple(f.join() if f is not None else None for f in forks)
        G = meta[4] if len(meta) > 4 and meta[3] == "grouped" else 1
        ctx.groups = G
        need_dx = ctx.needs_input_grad[0]
        cin_w = weight.shape[1]
        # grouped conv with 16-byte aligned groups: compact per-group operands
        # on group-aligned GEMM tiles (no block-diagonal zeros)
        gc = G > 1 and cin_w % 8 == 0 and (weight.shape[0] // G) % 8 == 0 and _GROUPED_COMPACT[0]
        link_in = getattr(x, "_mda_bnlink", None) if (need_dx and (G == 1 or gc) and _BNB_ON[0]) else None
        chpad = G == 1 and (not need_dx) and needs_channel_pad(cin_w)
        x_in = x
        x = pad_channels8(x) if chpad else _cl_bf16(x)
        N, Cin, H, W = x.shape
        Cout, _, KH, KW = weight.shape
        Ho = (H + 2 * pad - KH) // stride + 1
        Wo = (W + 2 * pad - KW) // stride + 1
        M = N * Ho * Wo
        K = KH * KW * Cin
        Kp = (K + 63) // 64 * 64
        KpT = (KH * KW * Cout + 63) // 64 * 64
        dev = x.device
        ctx.cin_keep = cin_w if chpad else 0
        ctx.kp_w = Kp  # the weight gradient runs dense over all Cin (keeps each group's block)
        packs = _ACTIVE[0]
        if gc:
            Kp = (KH * KW * cin_w + 63) // 64 * 64
            KpT = (KH * KW * (Cout // G) + 63) // 64 * 64
        ent = packs.lookup(weight, need_dx) if (packs is not None and not chpad and (G == 1 or gc)) else None
        pent = packs.lookup_pad(weight) if (packs is not None and chpad) else None
        if gc and ent is None:
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = torch.empty(Cin, KpT, dtype=torch.bfloat16, device=dev) if need_dx else None
            wc = weight.detach()
            if packs is not None and wc.is_contiguous() and wc.dtype == torch.float32:
                packs.register(weight, wf, wt, Cout, cin_w, KH, KW, Kp, KpT, groups=G)
            _ext.call("mda_pack_conv_weights_gc", wc.float().contiguous(), wf, wt, Cout, cin_w, KH, KW,
                      Kp, KpT, G)
        elif gc:
            wf, wt = ent["wf"], ent["wt"]
        elif G > 1:  # block-diagonal dense operands, packed per call (no multi-layer table)
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = torch.empty(Cin, KpT, dtype=torch.bfloat16, device=dev) if need_dx else None
            _ext.call("mda_pack_conv_weights_grouped", weight.detach().float().contiguous(), wf, wt,
                      Cout, Cin, KH, KW, Kp, KpT, G)
        elif chpad and pent is not None:  # packed for this step by PackCache.pack_all
            wf, wt = pent["wf"], None
        elif chpad:  # stem: forward operand with zero weights for the pad channels
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = None
            wc = weight.detach()
            if (packs is not None and wc.is_contiguous() and wc.dtype == torch.float32
                    and os.environ.get("MDA_PACK_EXTRAS", "1") != "0"):
                packs.register_pad(weight, wf, Cout, cin_w, Cin, KH, KW, Kp)
            _ext.call("mda_pack_conv_weights_pad", wc.contiguous(), wf, Cout, cin_w, Cin, KH, KW, Kp)
        elif ent is not None:  # packed for this step by PackCache.pack_all
            wf, wt = ent["wf"], ent["wt"]
        else:
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = torch.empty(Cin, KpT, dtype=torch.bfloat16, device=dev) if need_dx else None
            wc = weight.detach()
            if packs is not None and wc.is_contiguous() and wc.dtype == torch.float32:
                packs.register(weight, wf, wt, Cout, Cin, KH, KW, Kp, KpT)
            _ext.call("mda_pack_conv_weights", wc.contiguous(), wf, wt, Cout, Cin, KH, KW, Kp, KpT)
        from .hip_layers import conv_plan
        tile, splits = conv_plan(M, Cout, Kp)
        part = torch.empty(splits * M * Cout, dtype=torch.float32, device=dev) if splits > 1 else None
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=dev,
                        memory_format=torch.channels_last)
        ws = _ws(dev)
        stats = torch.empty(4, Cout, dtype=torch.float32, device=dev)  # mean, rstd, scale, shift
        res = _cl_bf16(residual) if residual is not None else None
        rv = getattr(residual, "_mda_vbn", None) if residual is not None else None
        if rv is not None and res is not residual:
            raise RuntimeError("a virtual residual must reach its consumer unchanged (bf16 NHWC)")
        if getattr(x, "_mda_vbn", None) is not None:
            raise RuntimeError("a virtual (un-applied) BN output reached a dense conv")
        # defer: a projection shortcut (act none) whose apply the block's
        # residual consumer performs
        defer = bool(defer) and (_BN_FUSED[0] or gc) and act == 0 \
            and residual is None and not want_preact and G == 1 and cbias is None
        ctx.vbn = None
        out = y if defer else torch.empty_like(y)
        pre = torch.empty_like(y) if want_preact else None
        if _BN_FUSED[0] or gc:
            # conv whose epilogue adds the BN sums into the stream's slot, then
            # apply with the finalize in its prologue (2 launches)
            reg = _region(Cout, dev)
            pend = _RIDE["apply"]
            rc = _ext.NOT_SERVED
            if (pend is not None and x_in is _RIDE["x"] and pend[0] == torch.cuda.current_stream()
                    and KH == 1 and KW == 1 and pad == 0 and G == 1 and splits == 1 and not gc):
                # a projection shortcut: conv1's parked BN apply rides in this launch
                rc = _ext.call("mda_conv1x1_bnacc_apply", x, wf, y, reg, N, H, W, Cin, Kp, Ho, Wo,
                               Cout, stride, *pend[1], ok=(0, _ext.NOT_SERVED))
                if rc == 0:
                    _RIDE["apply"] = None
                    _RIDE_COUNT[0] += 1
            if rc != 0:
                _flush_apply_ride()
                _ext.call("mda_conv_fwd_bnacc_g", x, wf, y, part, reg, N, H, W, Cin, Ho, Wo,
                          Cout, KH, KW, stride, pad, Kp, tile, splits, G if gc else 1)
            if defer:
                # no apply: the consumer's apply finalizes this BN (VirtualBN)
                ctx.vbn = VirtualBN(reg, gamma.detach(), beta.detach(), bn, stats)
            elif rv is not None:
                _ext.call("mda_bn_apply_fin_vr", y, reg, M, Cout, gamma.detach(), beta.detach(),
                          bn.running_mean, bn.running_var, stats, float(bn.momentum),
                          float(bn.eps), bn.num_batches_tracked, res, out, pre, act, rv.reg,
                          rv.gamma, rv.beta, rv.bn.running_mean, rv.bn.running_var, rv.stats,
                          float(rv.bn.momentum), float(rv.bn.eps), rv.bn.num_batches_tracked)
            else:
                args = (y, reg, M, Cout, gamma.detach(), beta.detach(), bn.running_mean,
                        bn.running_var, stats, float(bn.momentum), float(bn.eps),
                        bn.num_batches_tracked, res, out, pre, act)
                if (_RIDE["x"] is not None and x_in is _RIDE["x"] and _RIDE["apply"] is None
                        and res is None and pre is None):
                    # conv1 of an armed block: park its apply for the shortcut's launch
                    _RIDE["apply"] = (torch.cuda.current_stream(), args, (y, out))
                else:
                    _ext.call("mda_bn_apply_fin", *args)
        else:
            if rv is not None:
                raise RuntimeError("virtual residuals need the fused BN kernels (MDA_BN_FUSED=1)")
            # conv whose epilogue emits the BN statistics partials + finalize (2 launches)
            _ext.call("mda_conv_fwd_bnstats", x, wf, y, part, ws.partial, ws.partial.numel(), N, H,
                      W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kp, tile, splits, gamma.detach(),
                      beta.detach(), bn.running_mean, bn.running_var, stats[0], stats[1],
                      stats[2], stats[3], float(bn.momentum), float(bn.eps),
                      bn.num_batches_tracked)
            _ext.call("mda_bn_apply", y, stats[2], stats[3], res, out, pre, M, Cout, act)
        ctx.save_for_backward(x, wt, weight, gamma, beta, y, res, stats)
        ctx.meta = (N, Cin, H, W, Cout, Ho, Wo, KH, KW, stride, pad, Kp, KpT, act)
        ctx.vres = rv.stats if rv is not None else None
        ctx.gc = gc
        ctx.has_res = residual is not None
        ctx.link_in = link_in if (link_in is not None and link_in.C == Cin
                                  and link_in.M == N * H * W) else None
        # the residual's producer (a projection shortcut's BN: no activation, no
        # residual of its own, not forked): its backward sums come from ours
        rl = getattr(residual, "_mda_bnlink", None) if residual is not None else None
        ctx.res_link = rl if (rl is not None and _BNB_ON[0] and rl.act == 0 and rl.res is None
                              and rl.C == Cout and rl.M == M and forks[1] is None) else None
        # this layer's output, for its consumer's dgrad (no pre-activation
        # output: its gradient would join dz after the consumer's epilogue)
        ctx.bnlink = None
        if not want_preact and Cout <= 2048:
            ctx.bnlink = BnLink(y, res if act != 0 else None, stats, act, M, Cout, ctx.vres)
        _LAST_LINK[0] = ctx.bnlink
        _LAST_VBN[0] = ctx.vbn
        ctx.cbias = cbias is not None
        ctx.cbias_t = cbias
        if cbias is not None:
            # BN(y + b) == BN(y) in training; the running mean tracks mean(y) + b
            bn.running_mean.add_(cbias.detach(), alpha=float(bn.momentum))
        if want_preact:
            return out, pre
        return out, None

    @staticmethod
    def backward(ctx, dout, dpre):
        if _DUAL[0] is not None:
            return _conv_bn_backward_dual(ctx, dout, dpre)
        if ctx.kind == "dw":
            return _dw_backward(ctx, dout, dpre)
        x, wt, weight, gamma, beta, y, res, stats = ctx.saved_tensors
        N, Cin, H, W, Cout, Ho, Wo, KH, KW, stride, pad, Kp, KpT, act = ctx.meta
        M = N * Ho * Wo
        dev = y.device
        dout = _cl_bf16(dout) if dout is not None else None
        dpre = _cl_bf16(dpre) if dpre is not None else None
        # dgamma / dbeta straight into existing .grad buffers (flat views), else returned
        direct_gb = gamma.grad is not None and beta.grad is not None
        need_res = ctx.has_res and ctx.needs_input_grad[4]
        dy, dres, sums = _bn_bwd(dout, dpre, y, res, stats, gamma, beta, M, Cout, act, need_res,
                                 direct_gb, ctx.bnlink, getattr(ctx, "res_link", None),
                                 getattr(ctx, "vres", None))
        x_fork, res_fork = ctx.forks
        if need_res:
            dres = _fork_sum(res_fork, dres)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((N, Cin, H, W), dtype=torch.bfloat16, device=dev,
                             memory_format=torch.channels_last)
            from .hip_layers import conv_plan
            tile, splits = conv_plan(N * H * W, Cin, KpT)
            part = torch.empty(splits * N * H * W * Cin, dtype=torch.float32, device=dev) if splits > 1 else None
            other = x_fork.take() if x_fork is not None else None
            parks = other is None and x_fork is not None and x_fork.armed
            link = ctx.link_in
            folded = False
            if (parks and _MERGE_ON[0] and KH == 1 and KW == 1 and pad == 0 and stride > 1
                    and Cout % 64 == 0 and KpT == Cout and not ctx.gc and ctx.groups == 1
                    and x_fork.park(_DeferredDgrad(dy, wt, Cout, KpT, stride))):
                # projection shortcut: its input gradient is folded into the
                # other consumer's (conv1's) dgrad launch
                dx = None
                parks = False
            elif isinstance(other, _DeferredDgrad):
                reg = _region(Cin, dev) if link is not None else None
                rc = _ext.NOT_SERVED
                if other.stride == stride and tuple(other.dy.shape[2:]) == (Ho, Wo):
                    rc = _ext.call("mda_conv_dgrad_bnsum2", dy, wt, dx, N, H, W, Cin, Ho, Wo, Cout,
                                   KH, KW, stride, pad, KpT, link.y if reg is not None else None,
                                   link.res if reg is not None else None,
                                   link.stats if reg is not None else None,
                                   link.act if reg is not None else 0, reg,
                                   link.vres if reg is not None else None, other.dy, other.wt,
                                   other.cin2, other.kp2, ok=(0, _ext.NOT_SERVED))
                if rc == 0 and reg is not None:
                    link.arm(dx, reg)
                if rc == 0:
                    _MERGE_COUNT[0] += 1
                    folded = True
                else:
                    other = other.materialize((N, Cin, H, W))
            if dx is None or folded:
                pass
            elif ctx.gc:
                reg = _region(Cin, dev) if (link is not None and not parks and splits == 1) else None
                _ext.call("mda_conv_dgrad_bnsum_g", dy, wt, dx, part, other, N, H, W, Cin, Ho, Wo,
                          Cout, KH, KW, stride, pad, KpT, tile, splits,
                          link.y if reg is not None else None, link.res if reg is not None else None,
                          link.stats if reg is not None else None, link.act if reg is not None else 0,
                          reg, ctx.groups, link.vres if reg is not None else None, 0, 0)
                if reg is not None:
                    link.arm(dx, reg)
            elif link is not None and not parks and splits == 1:
                # dx is the whole output gradient of the BN layer that made x:
                # its backward sums come out of this epilogue (BnLink)
                reg = _region(Cin, dev)
                _ext.call("mda_conv_dgrad_bnsum_g", dy, wt, dx, part, other, N, H, W, Cin, Ho,
                          Wo, Cout, KH, KW, stride, pad, KpT, tile, splits, link.y, link.res,
                          link.stats, link.act, reg, 1, link.vres, 0, 0)
                link.arm(dx, reg)
            else:
                _ext.call("mda_conv_dgrad_res", dy, wt, dx, part, other, N, H, W, Cin, Ho, Wo,
                          Cout, KH, KW, stride, pad, KpT, tile, splits)
            if parks and x_fork.park(dx):
                dx = None
        dw = None
        if ctx.needs_input_grad[1]:
            Kw = ctx.kp_w
            sp = _wgrad_splits(M, Cout, Cin, KH, KW, Kw, H, W, stride, pad)
            direct_w = weight.grad is not None and weight.grad.is_contiguous()
            target = weight.grad if direct_w else torch.empty_like(weight, memory_format=torch.contiguous_format)

            def wg():
                _conv_wgrad(x, dy, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kw, sp,
                            direct_w, ctx.cin_keep, ctx.groups)
            wg()
            dw = None if direct_w else target
            if direct_w:
                notify_grad(weight)
        if direct_gb:
            notify_grad(gamma, beta)
        dgamma = None if direct_gb else sums[1].clone()
        dbeta = None if direct_gb else sums[0].clone()
        return dx, dw, dgamma, dbeta, dres, None, None, None, None, _cbias_grad(ctx), None, None


def _bn_bwd_dual(dout, dpre, y, res, stats, gamma, beta, M, C, act, need_res, link, res_link, vres):
    """Both gradient sets of :func:`_bn_bwd` in one launch (gridDim.y = 2):
    (dy, dres) as set-0 halves of stacked buffers."""
    D = _DUAL[0]
    dev = y.device
    if gamma.grad is None or beta.grad is None:
        raise RuntimeError("DOT single-pass backward: BN parameters need bound flat gradients")
    if not _BN_FUSED[0]:
        raise RuntimeError("DOT single-pass backward needs the fused BN kernels (MDA_BN_FUSED=1)")
    dual_full(dout)
    if dpre is not None:
        dual_full(dpre)
    _, dy = dual_alloc(tuple(y.shape), torch.bfloat16, dev)
    dres = dual_alloc(tuple(y.shape), torch.bfloat16, dev)[1] if need_res else None
    reg = link.take(dout) if link is not None else None
    rl = res_link if (need_res and res_link is not None and 256 % (C // 8) == 0) else None
    rreg = _region_pair(C, dev) if rl is not None else None
    ry, rst = (rl.y, rl.stats) if rl is not None else (None, None)
    rb = _region_bytes(C)
    if reg is not None and dpre is None:
        _ext.call("mda_bn_bwd_apply_reg", dout, None, y, res, stats, M, C, act, reg, dy, dres,
                  gamma.grad, beta.grad, None, ry, rst, rreg, vres, 2, M * C, D.gstride, rb)
    else:
        _ext.call("mda_bn_bwd_fused", dout, None, dpre, y, res, stats, M, C, act,
                  _region_pair(C, dev), _err_word(dev), dy, dres, gamma.grad, beta.grad, None, ry,
                  rst, rreg, vres, 2, M * C, D.gstride, rb)
    if rl is not None:
        rl.arm(dres, rreg)
    return dy, dres


def _conv_bn_backward_dual(ctx, dout, dpre):
    """:meth:`_ConvBNActTrain.backward` over two stacked cotangents (see
    :class:`_Dual`): the BN backward, dgrad (2N images, BN-sum epilogue with
    one region per set) and both weight gradients."""
    if ctx.kind == "dw":
        return _dw_backward_dual(ctx, dout, dpre)
    if ctx.gc or ctx.groups != 1:
        raise RuntimeError("DOT single-pass backward: grouped convs are not supported; set "
                           "RUNTIME.DOT_SINGLE_PASS=False")
    if ctx.cbias and (ctx.cbias_t.grad is None or not ctx.needs_input_grad[9]):
        # a conv bias in front of a training BN has an exactly zero gradient: both
        # sets keep their zeroed slots of the flat buffer (_cbias_grad)
        raise RuntimeError("DOT single-pass backward: a conv bias needs a bound flat gradient")
    if dout is None:
        raise RuntimeError("DOT single-pass backward: a layer output without a gradient")
    x, wt, weight, gamma, beta, y, res, stats = ctx.saved_tensors
    N, Cin, H, W, Cout, Ho, Wo, KH, KW, stride, pad, Kp, KpT, act = ctx.meta
    M = N * Ho * Wo
    dev = y.device
    if dout.dtype != torch.bfloat16 or not dout.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("DOT single-pass backward: gradient not bf16 channels_last")
    need_res = ctx.has_res and ctx.needs_input_grad[4]
    dy, dres = _bn_bwd_dual(dout, dpre, y, res, stats, gamma, beta, M, Cout, act, need_res,
                            ctx.bnlink, getattr(ctx, "res_link", None), getattr(ctx, "vres", None))
    x_fork, res_fork = ctx.forks
    if need_res:
        dres = _fork_sum(res_fork, dres)
    dx = None
    if ctx.needs_input_grad[0]:
        dx = dual_alloc((N, Cin, H, W), torch.bfloat16, dev)[1]
        from .hip_layers import conv_plan
        tile, splits = conv_plan(2 * N * H * W, Cin, KpT)
        part = torch.empty(splits * 2 * N * H * W * Cin, dtype=torch.float32, device=dev) \
            if splits > 1 else None
        other = x_fork.take() if x_fork is not None else None
        if isinstance(other, _DeferredDgrad):
            raise RuntimeError("a deferred shortcut dgrad reached the dual backward")
        if other is not None:
            dual_full(other)
        parks = other is None and x_fork is not None and x_fork.armed
        link = ctx.link_in
        if link is not None and not parks and splits == 1:
            reg = _region_pair(Cin, dev)
            _ext.call("mda_conv_dgrad_bnsum_g", dy, wt, dx, part, other, 2 * N, H, W, Cin, Ho, Wo,
                      Cout, KH, KW, stride, pad, KpT, tile, splits, link.y, link.res, link.stats,
                      link.act, reg, 1, link.vres, N * H * W, _region_bytes(Cin))
            link.arm(dx, reg)
        else:
            _ext.call("mda_conv_dgrad_res", dy, wt, dx, part, other, 2 * N, H, W, Cin, Ho, Wo,
                      Cout, KH, KW, stride, pad, KpT, tile, splits)
        if parks and x_fork.park(dx):
            dx = None
    if ctx.needs_input_grad[1]:
        if weight.grad is None or not weight.grad.is_contiguous():
            raise RuntimeError("DOT single-pass backward: conv weights need bound flat gradients")
        Kw = ctx.kp_w
        sp = _wgrad_splits(M, Cout, Cin, KH, KW, Kw, H, W, stride, pad)
        target = weight.grad

        def wg():  # both sets in one launch (x read by both)
            _conv_wgrad(x, dy, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kw, sp,
                        True, ctx.cin_keep, 1, 2, _DUAL[0].gstride)
        wg()
        notify_grad(weight)
    notify_grad(gamma, beta)
    return dx, None, None, None, dres, None, None, None, None, _cbias_grad(ctx), None, None


def _bn_train_forward(y, M, C, gamma, beta, bn, residual, act, want_preact, reg=None):
    """``reg``: a region the producer (the depthwise conv) already filled with
    the batch sums -- then no statistics pass."""
    dev = y.device
    ws = _ws(dev)
    stats = torch.empty(4, C, dtype=torch.float32, device=dev)  # mean, rstd, scale, shift
    res = _cl_bf16(residual) if residual is not None else None
    out = torch.empty_like(y)
    pre = torch.empty_like(y) if want_preact else None
    if _BN_FUSED[0] or reg is not None:
        if reg is None:
            reg = _region(C, dev)
            _ext.call("mda_bn_stats_acc", y, M, C, reg)
        _ext.call("mda_bn_apply_fin", y, reg, M, C, gamma.detach(), beta.detach(),
                  bn.running_mean, bn.running_var, stats, float(bn.momentum), float(bn.eps),
                  bn.num_batches_tracked, res, out, pre, act)
        return out, pre, res, stats
    _ext.call("mda_bn_stats2", y, M, C, ws.partial, gamma.detach(), beta.detach(),
              bn.running_mean, bn.running_var, stats[0], stats[1], stats[2], stats[3],
              float(bn.momentum), float(bn.eps), bn.num_batches_tracked)
    _ext.call("mda_bn_apply", y, stats[2], stats[3], res, out, pre, M, C, act)
    return out, pre, res, stats


def _bn_train_backward(ctx, dout, dpre, y, res, stats, gamma, beta, M, C, act):
    """-> (dy, dres, dgamma or None, dbeta or None); dgamma/dbeta go straight
    into bound flat-gradient views when present."""
    dout = _cl_bf16(dout) if dout is not None else None
    dpre = _cl_bf16(dpre) if dpre is not None else None
    direct_gb = gamma.grad is not None and beta.grad is not None
    dy, dres, sums = _bn_bwd(dout, dpre, y, res, stats, gamma, beta, M, C, act, res is not None,
                             direct_gb, getattr(ctx, "bnlink", None))
    if direct_gb:
        notify_grad(gamma, beta)
        return dy, dres, None, None
    return dy, dres, sums[1].clone(), sums[0].clone()


def _dw_forward(ctx, x, weight, gamma, beta, residual, stride, pad, act, bn, want_preact):
    ctx.kind = "dw"
    if getattr(x, "_mda_vbn", None) is not None:
        raise RuntimeError("a virtual (un-applied) BN output reached a depthwise conv")
    x = _cl_bf16(x)
    N, C, H, W = x.shape
    Ho = (H + 2 * pad - 3) // stride + 1
    Wo = (W + 2 * pad - 3) // stride + 1
    packs = _ACTIVE[0]
    ent = packs.lookup(weight, False) if packs is not None else None
    if ent is not None and ent["meta"][1] < 0:  # packed for this step by PackCache.pack_all
        wp = ent["wf"]
    else:
        wp = dw_pack(weight)
        wc = weight.detach()
        if packs is not None and wc.is_contiguous() and wc.dtype == torch.float32:
            packs.register_dw(weight, wp)
    y = torch.empty((N, C, Ho, Wo), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    M = N * Ho * Wo
    reg = None
    if _BN_FUSED[0]:
        # the depthwise kernel adds the BN batch sums of its output (no stats pass)
        reg = _region(C, x.device)
        _ext.call("mda_dw_fwd_bnacc", x, wp, y, reg, N, H, W, C, Ho, Wo, 3, 3, stride, pad)
    else:
        _ext.call("mda_dw_fwd", x, wp, None, None, None, y, None, N, H, W, C, Ho, Wo, 3, 3,
                  stride, pad, 0)
    out, pre, res, stats = _bn_train_forward(y, M, C, gamma, beta, bn, residual, act, want_preact,
                                             reg)
    ctx.save_for_backward(x, wp, weight, gamma, beta, y, res, stats)
    ctx.meta = (N, C, H, W, Ho, Wo, stride, pad, act)
    ctx.has_res = residual is not None
    # the depthwise layer's BN output feeds a pointwise conv (MobileNets): its
    # backward sums can come from that conv's dgrad epilogue (BnLink)
    ctx.bnlink = None if want_preact else BnLink(y, res if act != 0 else None, stats, act, M, C)
    _LAST_LINK[0] = ctx.bnlink
    return out, pre


def _dw_backward(ctx, dout, dpre):
    x, wp, weight, gamma, beta, y, res, stats = ctx.saved_tensors
    N, C, H, W, Ho, Wo, stride, pad, act = ctx.meta
    M = N * Ho * Wo
    dy, dres, dgamma, dbeta = _bn_train_backward(ctx, dout, dpre, y, res, stats, gamma, beta, M,
                                                 C, act)
    if not (ctx.has_res and ctx.needs_input_grad[4]):
        dres = None
    dx = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty((N, C, H, W), dtype=torch.bfloat16, device=y.device,
                         memory_format=torch.channels_last)
        _ext.call("mda_dw_dgrad", dy, wp, dx, N, H, W, C, Ho, Wo, 3, 3, stride, pad)
    dw = None
    if ctx.needs_input_grad[1]:
        nblk = _dw_wgrad_blocks(N, H, W, C, Ho, Wo, stride, pad)
        direct_w = weight.grad is not None and weight.grad.is_contiguous()
        target = weight.grad if direct_w else torch.empty_like(weight, memory_format=torch.contiguous_format)

        def wg():
            part = torch.empty(nblk * 9 * C, dtype=torch.float32, device=y.device)
            if direct_w and _WG_DEFER[0] is not None:
                # partials now, their sum in the backward's one multi-layer reduce
                _ext.call("mda_dw_wgrad", x, dy, part, None, N, H, W, C, Ho, Wo, 3, 3, stride,
                          pad, nblk, 1)
                _WG_DEFER[0].append([part.data_ptr(), target.data_ptr(), nblk, C, 1, 3, 3, 0, 1,
                                     0, -1])
                _WG_KEEP.append(part)
                return
            _ext.call("mda_dw_wgrad", x, dy, part, target, N, H, W, C, Ho, Wo, 3, 3, stride, pad,
                      nblk, 1 if direct_w else 0)
        wg()
        dw = None if direct_w else target
        if direct_w:
            notify_grad(weight)
    return dx, dw, dgamma, dbeta, dres, None, None, None, None, _cbias_grad(ctx), None, None


def _dw_backward_dual(ctx, dout, dpre):
    """:func:`_dw_backward` over two stacked cotangents (see :class:`_Dual`):
    both sets' BN backward in one launch, the depthwise dgrad over 2N images,
    and one weight-gradient partial launch per set (x read by both) into the
    two sets of the flat gradient."""
    if ctx.cbias and (ctx.cbias_t.grad is None or not ctx.needs_input_grad[9]):
        raise RuntimeError("DOT single-pass backward: a conv bias needs a bound flat gradient")
    if dout is None:
        raise RuntimeError("DOT single-pass backward: a layer output without a gradient")
    x, wp, weight, gamma, beta, y, res, stats = ctx.saved_tensors
    N, C, H, W, Ho, Wo, stride, pad, act = ctx.meta
    M = N * Ho * Wo
    dev = y.device
    if dout.dtype != torch.bfloat16 or not dout.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("DOT single-pass backward: gradient not bf16 channels_last")
    need_res = ctx.has_res and ctx.needs_input_grad[4]
    dy, dres = _bn_bwd_dual(dout, dpre, y, res, stats, gamma, beta, M, C, act, need_res,
                            getattr(ctx, "bnlink", None), None, None)
    dyf = dual_full(dy)
    dx = None
    if ctx.needs_input_grad[0]:
        full, dx = dual_alloc((N, C, H, W), torch.bfloat16, dev)
        _ext.call("mda_dw_dgrad", dyf, wp, full, 2 * N, H, W, C, Ho, Wo, 3, 3, stride, pad)
    if ctx.needs_input_grad[1]:
        if weight.grad is None or not weight.grad.is_contiguous():
            raise RuntimeError("DOT single-pass backward: conv weights need bound flat gradients")
        nblk = _dw_wgrad_blocks(N, H, W, C, Ho, Wo, stride, pad)
        for k in (0, 1):
            part = torch.empty(nblk * 9 * C, dtype=torch.float32, device=dev)
            dyk = dyf[k * N:(k + 1) * N]
            tgt = dual_ptr(weight.grad, k)
            if _WG_DEFER[0] is not None:
                _ext.call("mda_dw_wgrad", x, dyk, part, None, N, H, W, C, Ho, Wo, 3, 3, stride,
                          pad, nblk, 1)
                _WG_DEFER[0].append([part.data_ptr(), tgt, nblk, C, 1, 3, 3, 0, 1, 0, -1])
                _WG_KEEP.append(part)
            else:
                _ext.call("mda_dw_wgrad", x, dyk, part, tgt, N, H, W, C, Ho, Wo, 3, 3, stride,
                          pad, nblk, 1)
        notify_grad(weight)
    notify_grad(gamma, beta)
    return dx, None, None, None, dres, None, None, None, None, _cbias_grad(ctx), None, None


def _cbias_grad(ctx):
    """The gradient of a conv bias in front of a training BN is exactly zero
    (BN subtracts the batch mean).  A bias with a bound flat-gradient view
    (the training step) keeps its zeroed slot -- no kernel; otherwise a zero
    tensor, so ``.grad`` exists as with PyTorch's layers."""
    b = getattr(ctx, "cbias_t", None)
    if b is None or not ctx.needs_input_grad[9]:
        return None
    if b.grad is not None:
        notify_grad(b)
        return None
    return torch.zeros_like(b)


def pack_weights(weight, dgrad=True):
    """fp32 OIHW -> (bf16 [Cout][Kp], bf16 [Cin][KpT] or None, Kp, KpT)."""
    Cout, Cin, KH, KW = weight.shape
    Kp = (KH * KW * Cin + 63) // 64 * 64
    KpT = (KH * KW * Cout + 63) // 64 * 64
    wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=weight.device)
    wt = torch.empty(Cin, KpT, dtype=torch.bfloat16, device=weight.device) if dgrad else None
    _ext.call("mda_pack_conv_weights", weight.detach().float().contiguous(), wf, wt, Cout, Cin, KH,
              KW, Kp, KpT)
    return wf, wt, Kp, KpT


def conv_dgrad(dy, weight, x_shape, stride, pad):
    """Input gradient of conv2d (bf16 NHWC in/out) on the MFMA dgrad kernel."""
    from .hip_layers import conv_plan
    N, Cin, H, W = x_shape
    Cout, _, KH, KW = weight.shape
    dy = _cl_bf16(dy)
    Ho, Wo = dy.shape[2], dy.shape[3]
    _, wt, _, KpT = pack_weights(weight, True)
    dx = torch.empty((N, Cin, H, W), dtype=torch.bfloat16, device=dy.device,
                     memory_format=torch.channels_last)
    tile, splits = conv_plan(N * H * W, Cin, KpT)
    part = torch.empty(splits * N * H * W * Cin, dtype=torch.float32, device=dy.device) if splits > 1 else None
    _ext.call("mda_conv_dgrad", dy, wt, dx, part, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
              KpT, tile, splits)
    return dx


def conv_wgrad(x, dy, weight_shape, stride, pad):
    """Weight gradient of conv2d (fp32 OIHW) on the MFMA wgrad kernel."""
    Cout, Cin, KH, KW = weight_shape
    x = _cl_bf16(x)
    dy = _cl_bf16(dy)
    N, _, H, W = x.shape
    Ho, Wo = dy.shape[2], dy.shape[3]
    Kp = (KH * KW * Cin + 63) // 64 * 64
    M = N * Ho * Wo
    sp = _wgrad_splits(M, Cout, Cin, KH, KW, Kp, H, W, stride, pad)
    part = torch.empty(sp * Cout * Kp, dtype=torch.float32, device=x.device)
    out = torch.empty(weight_shape, dtype=torch.float32, device=x.device)
    _ext.call("mda_conv_wgrad", x, dy, part, out, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad,
              Kp, sp, 1.0, 0, 0, 1, 1, 0)
    return out


# ---------------------------------------------------------------------------
# Pre-activation networks (WRN, reference models/cifar/wrn.py:39-48): convs
# WITHOUT a following BN (residual add / activation fused into the conv
# epilogue) and BN + residual + activation on an existing tensor.

def conv_train_supported(x, conv) -> bool:
    """Dense conv (no BN after it) of a trainable layer on the native kernels."""
    if not (x.is_cuda and x.dim() == 4 and isinstance(conv, nn.Conv2d) and conv.groups == 1):
        return False
    if conv.bias is not None or conv.dilation != (1, 1) or conv.padding_mode != "zeros":
        return False
    if conv.stride[0] != conv.stride[1] or not isinstance(conv.padding, tuple) or conv.padding[0] != conv.padding[1]:
        return False
    if conv.kernel_size[0] != conv.kernel_size[1]:
        return False
    if conv.out_channels % 8 or (conv.in_channels % 8 and x.requires_grad):
        return False
    if not conv.weight.requires_grad:
        return False
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    return torch.is_grad_enabled()


def _act_mask(dout, out, act):
    if act == 1:
        return torch.where(out > 0, dout, torch.zeros((), dtype=dout.dtype, device=dout.device))
    if act == 2:
        return torch.where((out > 0) & (out < 6), dout, torch.zeros((), dtype=dout.dtype, device=dout.device))
    return dout


class _ConvTrain(torch.autograd.Function):
    """out = act(conv(x) + residual): ONE conv launch (residual and activation in
    the epilogue); backward = activation mask (if any) + dgrad + wgrad."""

    @staticmethod
    def forward(ctx, x, weight, residual, meta, want_preact):
        ctx.set_materialize_grads(False)
        stride, pad, act = meta
        need_dx = ctx.needs_input_grad[0]
        cin_w = weight.shape[1]
        chpad = (not need_dx) and needs_channel_pad(cin_w)
        x = pad_channels8(x) if chpad else _cl_bf16(x)
        N, Cin, H, W = x.shape
        Cout, _, KH, KW = weight.shape
        Ho = (H + 2 * pad - KH) // stride + 1
        Wo = (W + 2 * pad - KW) // stride + 1
        M = N * Ho * Wo
        Kp = (KH * KW * Cin + 63) // 64 * 64
        KpT = (KH * KW * Cout + 63) // 64 * 64
        dev = x.device
        packs = _ACTIVE[0]
        ent = packs.lookup(weight, need_dx) if (packs is not None and not chpad) else None
        if chpad:
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = None
            _ext.call("mda_pack_conv_weights_pad", weight.detach().contiguous(), wf, Cout, cin_w,
                      Cin, KH, KW, Kp)
        elif ent is not None:
            wf, wt = ent["wf"], ent["wt"]
        else:
            wf = torch.empty(Cout, Kp, dtype=torch.bfloat16, device=dev)
            wt = torch.empty(Cin, KpT, dtype=torch.bfloat16, device=dev) if need_dx else None
            wc = weight.detach()
            if packs is not None and wc.is_contiguous() and wc.dtype == torch.float32:
                packs.register(weight, wf, wt, Cout, Cin, KH, KW, Kp, KpT)
            _ext.call("mda_pack_conv_weights", wc.contiguous(), wf, wt, Cout, Cin, KH, KW, Kp, KpT)
        from .hip_layers import conv_plan
        tile, splits = conv_plan(M, Cout, Kp)
        part = torch.empty(splits * M * Cout, dtype=torch.float32, device=dev) if splits > 1 else None
        res = _cl_bf16(residual) if residual is not None else None
        out = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=dev,
                          memory_format=torch.channels_last)
        pre = torch.empty_like(out) if (want_preact or act != 0) else None
        _ext.call("mda_conv_fwd", x, wf, None, None, res, out, pre, part, N, H, W, Cin, Ho, Wo,
                  Cout, KH, KW, stride, pad, Kp, act, tile, splits)
        ctx.save_for_backward(x, wt, weight, pre if act != 0 else None)
        ctx.meta = (N, Cin, H, W, Cout, Ho, Wo, KH, KW, stride, pad, Kp, KpT, act)
        ctx.cin_keep = cin_w if chpad else 0
        ctx.has_res = residual is not None
        return out, (pre if want_preact else None)

    @staticmethod
    def backward(ctx, dout, dpre):
        x, wt, weight, pre = ctx.saved_tensors
        N, Cin, H, W, Cout, Ho, Wo, KH, KW, stride, pad, Kp, KpT, act = ctx.meta
        M = N * Ho * Wo
        dev = x.device
        dz = None
        if dout is not None and pre is not None and pre.numel() % 8 == 0 \
                and pre.is_contiguous(memory_format=torch.channels_last):
            # act' * dout (+ dpre) in one native launch
            dz = torch.empty_like(pre)
            _ext.call("mda_act_bwd", _cl_bf16(dout), pre, _cl_bf16(dpre) if dpre is not None else None,
                      dz, pre.numel(), act)
        else:
            if dout is not None:
                dz = _act_mask(_cl_bf16(dout), pre, act)
            if dpre is not None:
                dz = _cl_bf16(dpre) if dz is None else dz + _cl_bf16(dpre)
        dz = _cl_bf16(dz)
        dres = dz if (ctx.has_res and ctx.needs_input_grad[2]) else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((N, Cin, H, W), dtype=torch.bfloat16, device=dev,
                             memory_format=torch.channels_last)
            from .hip_layers import conv_plan
            tile, splits = conv_plan(N * H * W, Cin, KpT)
            part = torch.empty(splits * N * H * W * Cin, dtype=torch.float32, device=dev) if splits > 1 else None
            _ext.call("mda_conv_dgrad", dz, wt, dx, part, N, H, W, Cin, Ho, Wo, Cout, KH, KW,
                      stride, pad, KpT, tile, splits)
        dw = None
        if ctx.needs_input_grad[1]:
            sp = _wgrad_splits(M, Cout, Cin, KH, KW, Kp, H, W, stride, pad)
            direct_w = weight.grad is not None and weight.grad.is_contiguous()
            target = weight.grad if direct_w else torch.empty_like(weight, memory_format=torch.contiguous_format)

            def wg():
                _conv_wgrad(x, dz, target, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, Kp, sp,
                            direct_w, ctx.cin_keep, 1)
            wg()
            dw = None if direct_w else target
            if direct_w:
                notify_grad(weight)
        return dx, dw, dres, None, None


def conv_act_train(x, conv, act, residual, want_preact):
    out, pre = _ConvTrain.apply(x, conv.weight, residual,
                                (conv.stride[0], conv.padding[0], _ACT[act]), bool(want_preact))
    return out, pre


def bn_train_supported(x, bn) -> bool:
    if not (x.is_cuda and x.dim() == 4 and isinstance(bn, nn.BatchNorm2d)):
        return False
    if not bn.training or not bn.track_running_stats or bn.momentum is None:
        return False
    if bn.weight is None or bn.bias is None or x.shape[1] % 8 or x.shape[1] > 2048:
        return False
    if x.dtype != torch.bfloat16 and not (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    return torch.is_grad_enabled()


class _BNActTrain(torch.autograd.Function):
    """Training BN (+ residual) (+ activation) of an existing activation: batch
    statistics (+ running-stat update) and apply, 3 launches; backward 3."""

    @staticmethod
    def forward(ctx, x, gamma, beta, residual, bn, act, want_preact):
        ctx.set_materialize_grads(False)
        y = _cl_bf16(x)
        N, C, H, W = y.shape
        M = N * H * W
        out, pre, res, stats = _bn_train_forward(y, M, C, gamma, beta, bn, residual, act,
                                                 want_preact)
        ctx.save_for_backward(y, res, stats, gamma, beta)
        ctx.meta = (M, C, act)
        ctx.has_res = residual is not None
        return out, pre

    @staticmethod
    def backward(ctx, dout, dpre):
        y, res, stats, gamma, beta = ctx.saved_tensors
        M, C, act = ctx.meta
        dy, dres, dgamma, dbeta = _bn_train_backward(ctx, dout, dpre, y, res, stats, gamma, beta,
                                                     M, C, act)
        if not (ctx.has_res and ctx.needs_input_grad[3]):
            dres = None
        return dy, dgamma, dbeta, dres, None, None, None


def bn_act_train(x, bn, act, residual, want_preact):
    out, pre = _BNActTrain.apply(x, bn.weight, bn.bias, residual, bn, _ACT[act], bool(want_preact))
    return out, pre


# ---------------------------------------------------------------------------
# Frozen conv + TRAIN-mode BN without autograd: the OFD teacher (reference
# distillers/OFD.py:114-121 keeps the teacher's BN in training mode, so its
# forward normalises with batch statistics and updates running statistics).
# MIOpen's train-mode BN replayed from a hipGraph in bf16 went non-finite run
# to run (profiles/r1_ofd_graph_ab.md); these kernels are capture-safe.

def trainbn_nograd_supported(x, conv, bn) -> bool:
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad):
        return False
    if not (x.is_cuda and x.dim() == 4 and isinstance(conv, nn.Conv2d) and conv.groups == 1):
        return False
    if bn is None or not bn.training or not bn.track_running_stats or bn.momentum is None:
        return False
    if conv.bias is not None or conv.dilation != (1, 1) or conv.padding_mode != "zeros":
        return False
    if conv.stride[0] != conv.stride[1] or not isinstance(conv.padding, tuple) or conv.padding[0] != conv.padding[1]:
        return False
    if conv.kernel_size[0] != conv.kernel_size[1] or conv.out_channels % 8 or conv.out_channels > 2048:
        return False
    return x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                         and torch.get_autocast_dtype("cuda") == torch.bfloat16)


@torch.no_grad()
def conv_trainbn_nograd(x, conv, bn, act, residual, want_preact):
    from .hip_layers import conv_bn_act as conv_infer
    y, _ = conv_infer(x, conv, None, "none", None, False)  # packed once per weight version
    N, C, Ho, Wo = y.shape
    gamma = bn.weight if bn.weight is not None else torch.ones(C, device=y.device)
    beta = bn.bias if bn.bias is not None else torch.zeros(C, device=y.device)
    out, pre, _, _ = _bn_train_forward(y, N * Ho * Wo, C, gamma, beta, bn, residual, _ACT[act],
                                       want_preact)
    return out, pre


def conv_bn_act_train(x, conv, bn, act, residual, want_preact, fork=None, res_fork=None,
                      defer_apply=False, private=False):
    """``fork``: the :class:`GradFork` of ``x`` (another consumer of x sums
    its gradient into this layer's dgrad, or vice versa); ``res_fork``: the
    fork of ``residual`` (identity shortcut).  ``defer_apply``: return the raw
    conv output as a :class:`VirtualBN` (the caller guarantees its one
    consumer is a native conv + BN that takes it as ``residual``)."""
    meta = (conv.stride[0], conv.padding[0], _ACT[act])
    if is_depthwise(conv):
        meta = meta + ("dw",)
        fork = res_fork = None
    elif conv.groups != 1:
        meta = meta + ("grouped", conv.groups)
    if residual is None:
        res_fork = None
    _LAST_LINK[0] = None
    _LAST_VBN[0] = None
    defer = defer_apply if (defer_apply and conv.bias is None) else False
    out, pre = _ConvBNActTrain.apply(x, conv.weight, bn.weight, bn.bias, residual, meta, bn,
                                     bool(want_preact), (fork, res_fork), conv.bias, defer,
                                     bool(private))
    link, _LAST_LINK[0] = _LAST_LINK[0], None
    vbn, _LAST_VBN[0] = _LAST_VBN[0], None
    if link is not None:
        out._mda_bnlink = link
    if vbn is not None:
        out._mda_vbn = vbn
    return out, pre
