"""The training step: forward (teacher || student) -> losses -> backward ->
gradient all-reduce -> fused optimizer update -> on-device metrics.

This is the hot loop of the reference (`engine/trainer.py:257-321` base,
`:412-461` DOT, CRD variants), restructured for MI355X:

* **No host syncs.**  Losses, top-1/top-5 counts and sample counts are
  accumulated in device tensors (:class:`DeviceMeters`) and read once per
  log interval; the reference does an all-gather of predictions and four
  blocking ``.cpu()`` all-reduces every iteration.
* **hipGraph capture.**  After a few eager warm-up steps the whole step
  (forward, backward, optimizer, metric update) is captured once with
  ``torch.cuda.graph`` and replayed; only the batch copy into the static
  input buffers and the graph launch remain on the host.  At batch 64 per
  GPU a CIFAR distillation step is ~300-600 small kernels, so this removes
  the dominant (launch-bound) cost.  With world > 1 the collectives stay
  outside the captured graphs (forward/backward graph -> RCCL all-reduce ->
  optimizer graph); with ``DIST.GRAPH_COMM=events`` (the default) each
  bucket's all-reduce is launched right after the replay, behind an event
  node of the captured backward, so it overlaps the remaining backward.
* **Flat parameters** (:mod:`.optim`) -> one all-reduce, one optimizer launch.
* **DOT** runs its two backwards into the two halves of one ``[2, n]``
  gradient buffer and reduces both with one collective (fixes SURVEY D4).
"""
from __future__ import annotations

import contextlib

import os

# zero fills and the stem image pad ride in the weight-pack launch (A/B knob)
_PACK_EXTRAS = os.environ.get("MDA_PACK_EXTRAS", "1") != "0"

import torch

from ..parallel import GradReducer, get_world_size
from ..runtime.streams import join_branches
from .optim import FlatParams, FlatDOT, build_optimizer


def topk_rank(preds: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Position of the target class in a stable descending sort of ``preds``.

    Classes ranked before the target: strictly larger logits, plus equal
    logits at a lower class index (the order ``topk`` returns ties in), so a
    tie with the target -- common with bf16 logits -- is not a free hit.
    ``rank < k`` is the top-k hit test; computed with compares + a row sum
    instead of ``topk`` (whose multi-block ROCm path is not capture-safe and
    needs a sort), so it lives inside the captured step.
    """
    tgt = target.reshape(-1, 1)
    t = preds.gather(1, tgt)
    idx = torch.arange(preds.shape[1], device=preds.device).reshape(1, -1)
    return ((preds > t) | ((preds == t) & (idx < tgt))).sum(1)


def autograd_reachable(roots) -> set:
    """ids of the leaf tensors whose AccumulateGrad node is reachable from
    ``roots``' autograd graphs (a graph walk; nothing is computed)."""
    out, seen = set(), set()
    keep = []  # hold every visited node wrapper: a freed wrapper's id() gets reused
    stack = [r.grad_fn for r in roots if r.grad_fn is not None]
    while stack:
        fn = stack.pop()
        if fn is None or id(fn) in seen:
            continue
        seen.add(id(fn))
        keep.append(fn)
        v = getattr(fn, "variable", None)
        if v is not None:
            out.add(id(v))
        for nxt, _ in fn.next_functions:
            if nxt is not None:
                stack.append(nxt)
    return out


class DeviceMeters:
    """Loss sums and top-k hit counts kept on device; synced on demand."""

    def __init__(self, device, loss_keys):
        self.device = device
        self.loss_keys = list(loss_keys)
        # [sum(loss total), per-key..., top1 hits, top5 hits, samples, steps]
        self.buf = torch.zeros(len(self.loss_keys) + 5, dtype=torch.float64, device=device)

    def update(self, preds, target, losses: dict):
        if self._native(preds, losses):
            from ..ops import _ext
            ls = [losses[k].detach().reshape(()) for k in self.loss_keys]
            ls = [v if v.dtype == torch.float32 else v.float() for v in ls]
            ptrs = ls + [None] * (4 - len(ls))
            p = preds.detach()
            if p.dtype not in (torch.float32, torch.bfloat16):
                p = p.float()
            _ext.call("mda_meters_update", 0 if p.dtype == torch.float32 else 1, p.contiguous(),
                      target.contiguous(), p.shape[0], p.shape[1], *ptrs, len(ls), self.buf)
            return
        b = self.buf
        total = None
        for i, k in enumerate(self.loss_keys):
            v = losses[k].detach().double().reshape(())
            b[1 + i] += v
            total = v if total is None else total + v
        b[0] += total
        n = len(self.loss_keys)
        rank = topk_rank(preds.detach(), target)
        b[n + 1] += (rank < 1).sum().double()
        b[n + 2] += (rank < 5).sum().double()
        b[n + 3] += float(target.shape[0])
        b[n + 4] += 1.0

    def _native(self, preds, losses) -> bool:
        from ..ops.backend import hip_enabled_for
        return (len(self.loss_keys) <= 4 and preds.dim() == 2 and hip_enabled_for(preds)
                and all(losses[k].numel() == 1 for k in self.loss_keys))

    def reset(self):
        self.buf.zero_()

    def summary(self, reduce: bool = True) -> dict:
        """Global (all-rank) averages; one small all-reduce + one D2H copy."""
        from ..parallel import dist_fn
        t = self.buf.clone()
        if reduce:
            t = dist_fn.reduce(t, "sum")
        t = t.cpu()
        n = len(self.loss_keys)
        steps = max(t[n + 4].item(), 1.0)
        world = get_world_size() if reduce else 1
        samples = max(t[n + 3].item(), 1.0)
        out = {"loss": t[0].item() / steps / world}
        for i, k in enumerate(self.loss_keys):
            out[k] = t[1 + i].item() / steps / world
        out["top1"] = 100.0 * t[n + 1].item() / samples
        out["top5"] = 100.0 * t[n + 2].item() / samples
        out["samples"] = samples
        return out


def _autocast(device, dtype):
    if device.type == "cuda" and dtype in (torch.bfloat16, torch.float16):
        return torch.autocast(device_type="cuda", dtype=dtype, cache_enabled=False)
    return contextlib.nullcontext()


def _multi_copy(dst, src):
    """``dst[i].copy_(src[i])`` for same-shape, same-dtype, same-layout device
    tensors in ONE launch (ops/csrc/optim.hip mda_multi_copy); otherwise (or
    beyond 16 pairs) torch._foreach_copy_ (one blit per tensor)."""
    ok = (0 < len(dst) <= 16 and all(
        d.is_cuda and s.is_cuda and d.dtype == s.dtype and d.shape == s.shape
        and d.stride() == s.stride() and d.is_contiguous(memory_format=_fmt(d))
        for d, s in zip(dst, src)))
    if ok:
        from ..ops import _ext
        if _ext.available():
            tab = torch.tensor([[s.data_ptr(), d.data_ptr(), d.numel() * d.element_size()]
                                for d, s in zip(dst, src)], dtype=torch.int64)
            _ext.call("mda_multi_copy", tab, len(dst))
            return
    torch._foreach_copy_(dst, src)


def _fmt(t):
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return torch.channels_last
    return torch.contiguous_format


def _to_channels_last(module):
    for m in module.modules():
        for name, p in list(m.named_parameters(recurse=False)):
            if p.dim() == 4:
                p.data = p.data.contiguous(memory_format=torch.channels_last)
    return module


class TrainStep:
    """One optimisation step of a distiller; see module docstring.

    ``batch_keys``: names of the per-step tensors passed to the distiller
    besides ``epoch`` (``image, target`` or CRD's ``image, target, index,
    contrastive_index``).
    """

    def __init__(self, distiller, cfg, device, trainer: str = "base", use_graph: bool = False,
                 dtype: torch.dtype = torch.float32, batch_keys=("image", "target"),
                 channels_last: bool = None, warmup_eager: int = 3):
        self.distiller = distiller
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type == "cuda":
            from ..runtime import streams as _streams
            _streams.renew(self.device)  # same stream layout as a fresh process
        self.trainer = trainer
        self.is_dot = trainer in ("dot", "crd_dot")
        self.dtype = dtype
        self.batch_keys = tuple(batch_keys)
        if channels_last is None:
            channels_last = self.device.type == "cuda"
        self.channels_last = channels_last
        if channels_last:
            _to_channels_last(distiller)
        self.world = get_world_size()
        # EXPERIMENT.DETERMINISTIC: fixed-order reductions on the native path
        # (ops/hip_train.py set_deterministic) and PyTorch's deterministic algorithms
        self.deterministic = bool(cfg.EXPERIMENT.get("DETERMINISTIC", False))
        if self.device.type == "cuda":
            from ..ops import hip_train as _ht
            _ht.set_deterministic(self.deterministic)
            if self.deterministic:
                torch.backends.cudnn.deterministic = True
        self.flat = FlatParams(distiller.get_learnable_parameters(), 2 if self.is_dot else 1)
        self.opt = build_optimizer(cfg, self.flat, grad_scale=1.0 / self.world, trainer=trainer)
        self.use_graph = (bool(use_graph) and self.device.type == "cuda"
                          and getattr(distiller, "graph_capturable", True))
        if self.use_graph and not self.deterministic:
            # MIOpen find mode: algorithms are chosen during the eager warm-up
            # steps, so nothing is searched or JIT-built inside a capture
            torch.backends.cudnn.benchmark = True
        if self.world > 1 and getattr(distiller, "collective_in_forward", False):
            self.use_graph = False  # its collectives must not be captured
        if self.world > 1 and bool(cfg.DIST.get("BROADCAST_INIT", True)):
            # DDP's constructor broadcast (reference tools/train.py:86, site C2):
            # every parameter and buffer of the distiller from rank 0
            from ..parallel import broadcast_initial_state
            broadcast_initial_state(distiller, self.flat)
        self.graph_comm = self._graph_comm_mode(cfg)
        self.reducer = GradReducer(self.flat, bucket_mb=float(cfg.DIST.BUCKET_MB),
                                   overlap=True, wire_dtype=cfg.DIST.GRAD_DTYPE)
        self.epoch_t = torch.zeros((), dtype=torch.float32, device=self.device)
        self._epoch = None
        self.meters = None
        self.warmup_eager = max(1, int(warmup_eager))
        self.steps_done = 0
        self._graphs = None
        self._static_img = None  # the captured step's input image (pack-table extras)
        self._static = None
        self._dot_ready = not self.is_dot
        self._reach_ready = False
        self._units = {}
        self._packs = None
        self._dual = None  # DOT: (fwd, kd-bwd, ce-bwd, opt, upd graphs, side stream, event)
        self.dot_dual = self.is_dot and bool(cfg.RUNTIME.get("DOT_DUAL_STREAM", True))
        self.dot_single = self.is_dot and self._dot_single_ok(cfg)
        la = cfg.RUNTIME.get("TEACHER_LOOKAHEAD", "auto")
        la = la.lower() if isinstance(la, str) else bool(la)
        self.lookahead = "auto" if la == "auto" else la in (True, "true", "1", "on")
        self._pipe = None       # (teacher-only graph, TeacherFeed) when the look-ahead is captured
        self._static_next = None
        self._x_for = None      # the image tensor whose teacher outputs the feed holds
        self._la_misses = 0     # consecutive look-ahead steps without a next batch
        # the look-ahead teacher as its own graph on the teacher stream (see
        # runtime/streams.py::TeacherFeed.capture_pipe) instead of a branch of
        # the step graph
        self.teacher_split = str(cfg.RUNTIME.get("TEACHER_GRAPH", "split")).lower() == "split"
        if getattr(distiller, "_teacher_train_bn", False):
            # a train-mode teacher (OFD.TEACHER_TRAIN_BN) keeps its look-ahead a
            # branch of the step graph: as a graph of its own, the SECOND replay
            # of the step graph finds garbage BN sums in a connector BN
            # (running_var inf / NaN losses, scripts/debug/ofd_lookahead_nan.py;
            # only with the fused BN regions, teacher graph replayed or not);
            # cause not found
            self.teacher_split = False
        self.teacher_first = bool(cfg.RUNTIME.get("TEACHER_FIRST", True))
        self._tsplit = None     # (graph, T list, X list, stream, teacher-done event, copy-done event)
        self._tp_inflight = False
        self.wgrad_defer = self.device.type == "cuda" and bool(cfg.RUNTIME.get("WGRAD_DEFER", True))

    def _graph_comm_mode(self, cfg):
        """How the gradient all-reduce meets the captured step at world > 1.

        ``False`` (split): fwd+bwd graph -> eager bucketed all-reduce -> optimizer
        graph.  ``"events"`` (auto): the same two graphs, but the captured
        backward records one external event per gradient bucket and the
        all-reduces are enqueued right after the replay launch on a comm
        stream, each behind its bucket's event, so they overlap the rest of the
        backward (GradReducer.arm_capture).  (An all-reduce captured inside the
        step graph needs a multi-branch graph, slow on ROCm's executor: not
        offered.)
        """
        if self.world <= 1 or not self.use_graph:
            return False
        mode = str(cfg.DIST.get("GRAPH_COMM", "auto")).lower()
        if mode in ("events", "auto"):
            return "events"
        if mode == "split":
            return False
        raise ValueError(f"DIST.GRAPH_COMM={mode!r}: expected auto | events | split")

    # ------------------------------------------------------------------
    def set_epoch(self, epoch: float) -> None:
        if epoch != self._epoch:
            self._epoch = epoch
            self.epoch_t.fill_(float(epoch))

    def set_lr(self, lr: float) -> None:
        self.opt.set_lr(lr)

    def _prep(self, batch: dict) -> dict:
        out = {}
        for k in self.batch_keys:
            v = batch[k]
            if k == "image":
                v = v.to(self.device, non_blocking=True).float() if v.device != self.device else v
                if self.channels_last and v.dim() == 4:
                    v = v.contiguous(memory_format=torch.channels_last)
            else:
                v = v.to(self.device, non_blocking=True)
            out[k] = v
        return out

    def _prep_image(self, v):
        v = v.to(self.device, non_blocking=True).float() if v.device != self.device else v
        if self.channels_last and v.dim() == 4:
            v = v.contiguous(memory_format=torch.channels_last)
        return v

    def _forward(self, b: dict):
        with _autocast(self.device, self.dtype):
            preds, losses = self.distiller(epoch=self.epoch_t, **b)
        if self.meters is None:
            self.meters = DeviceMeters(self.device, sorted(losses.keys()))
        return preds, losses

    def _unit(self, v):
        key = (v.dtype, v.device, tuple(v.shape))
        u = self._units.get(key)
        if u is None:
            u = self._units[key] = torch.ones_like(v)
            if u.numel() == 1:
                from ..ops.losses import register_unit_seed
                register_unit_seed(u)
        return u

    # module types whose whole backward runs on the native kernels that carry
    # two stacked cotangents (ops/hip_train.py _Dual): the CIFAR ResNets
    # (Bottleneck ResNets are left out: no test covers their dual backward)
    _DOT_SINGLE_MODULES = frozenset({"ResNet", "BasicBlock", "VGG", "MobileNetV2", "InvertedResidual",
                                     "LinearBottleNeck", "Conv2d", "BatchNorm2d", "Linear", "ReLU",
                                     "ReLU6", "Sequential", "ModuleList", "Identity", "Stage",
                                     "AdaptiveAvgPool2d", "AvgPool2d", "MaxPool2d"})

    def _dot_single_ok(self, cfg) -> bool:
        """``RUNTIME.DOT_SINGLE_PASS`` (auto | True | False): DOT's KD and task
        backwards as ONE pass over two stacked cotangents (reference
        trainer.py:425-432 runs two).  auto = the trainer is plain DOT, the
        student's modules are all on the list above and the HIP kernels run."""
        v = cfg.RUNTIME.get("DOT_SINGLE_PASS", "auto")
        v = v.lower() if isinstance(v, str) else bool(v)
        if v in (False, "false", "0", "off") or self.trainer != "dot" or self.device.type != "cuda":
            return False
        if self.dtype != torch.bfloat16:
            return False  # the native training kernels are the bf16 path
        student = getattr(self.distiller, "student", None)
        if student is None:
            return False
        from ..ops.backend import hip_enabled_for
        from ..ops import hip_train
        if not (hip_enabled_for(self.flat.data) and hip_train._BN_FUSED[0]):
            return False
        from ..ops.nn import MaxPool2d as NativeMaxPool
        for m in student.modules():
            name = type(m).__name__
            if name not in self._DOT_SINGLE_MODULES:
                return False
            if name == "Conv2d" and m.groups != 1:
                if not m.groups == m.in_channels == m.out_channels:
                    return False  # grouped
                if v == "auto":
                    # depthwise students run the single pass correctly but slower:
                    # Tiny-ImageNet R18 -> MV2 19.6 vs 18.2 ms/step for the two
                    # backwards on two streams; DOT_SINGLE_PASS=True forces it
                    return False
            if name == "MaxPool2d" and not isinstance(m, NativeMaxPool):
                return False  # torch's max pool: its backward cannot carry two sets
        return True

    def _dot_single_backward(self, losses):
        """Both DOT gradient sets from one backward (``self.dot_single``): the
        bound set is the KD one, the CE set sits ``gstride`` floats away."""
        from ..ops import hip_train
        self.flat.bind_grads(1)
        g = self.flat.grads
        gstride = (g[0].data_ptr() - g[1].data_ptr()) // g.element_size()
        terms = [losses["loss_kd"], losses["loss_ce"]]
        hip_train.set_dual(gstride)
        try:
            torch.autograd.backward(terms, [self._unit(v) for v in terms])
        finally:
            hip_train.set_dual(None)

    def _dot_reachability(self, losses):
        """Which params receive task / KD gradients (DOT's momentum branches)."""
        ps = self.flat.params
        rt = autograd_reachable([losses["loss_ce"]])
        rk = autograd_reachable([losses["loss_kd"]])
        self.opt.set_reachability([id(p) in rt for p in ps], [id(p) in rk for p in ps])
        self._dot_ready = True

    def _grad_reachability(self, losses):
        """Params no loss reaches get no update (torch.optim skips grad-None params)."""
        r = autograd_reachable([v for v in losses.values() if v.requires_grad])
        self.opt.set_active([id(p) in r for p in self.flat.params])
        self._reach_ready = True

    def _fwd_bwd(self, b: dict, overlap_comm):
        preds, losses = self._fwd(b)
        deferred = self._arm_wgrad_defer()
        # DOT's single pass writes both gradient sets of a parameter together:
        # its buckets launch both sets from the same events
        events = overlap_comm == "events" and (not self.is_dot or self.dot_single)
        try:
            if self.is_dot and self.dot_single:
                if events:
                    from ..ops import hip_train
                    self.reducer.sets = (0, 1)
                    self.reducer.arm_capture(hip_train.flush_wgrad_reduces if deferred else None)
                    events = "armed"
                elif self.world > 1 and not torch.cuda.is_current_stream_capturing():
                    self.reducer.calibrate()  # counts for a later events capture
                self._dot_single_backward(losses)
            elif self.is_dot:
                self.flat.bind_grads(1)
                losses["loss_kd"].backward(retain_graph=True)
                self.flat.bind_grads(0)
                losses["loss_ce"].backward()
            else:
                if events:
                    from ..ops import hip_train
                    # a bucket's deferred weight-gradient reductions are flushed
                    # before its event, so the event marks final gradients
                    self.reducer.arm_capture(hip_train.flush_wgrad_reduces if deferred else None)
                    events = "armed"
                elif overlap_comm:
                    self.reducer.arm()
                # backward of the loss terms with unit seeds straight into each term
                # (no sum node, no per-step fill kernels)
                terms = [v for v in losses.values() if v.requires_grad]
                if terms:
                    torch.autograd.backward(terms, [self._unit(v) for v in terms])
        except BaseException:
            if events == "armed":
                self.reducer.abort_capture()
            raise
        finally:
            if self.is_dot and self.dot_single and events != "armed":
                self.reducer.end_calibration()
            self._flush_wgrad_defer(deferred)
            join_branches()
        if events == "armed":
            self.reducer.finish_capture()
        self._post_backward()
        feed = self.distiller.__dict__.get("_teacher_feed")
        if feed is not None:
            feed.finish()  # look-ahead: join the next batch's teacher forward
        return preds, losses

    def _arm_wgrad_defer(self) -> bool:
        """While a backward is being captured, defer every layer's split
        reduction to one multi-layer launch at the end of the backward
        (``hip_train.set_wgrad_defer``); each weight-gradient GEMM then rides
        in the launch of the next BN-backward apply (mda_conv_wgrad_nored_bn)."""
        if not (self.wgrad_defer and torch.cuda.is_current_stream_capturing()):
            return False
        from ..ops import hip_train
        hip_train.set_wgrad_defer(True)
        return True

    def _flush_wgrad_defer(self, armed: bool) -> None:
        if armed:
            from ..ops import hip_train
            try:
                hip_train.flush_wgrad_reduces()
            finally:
                hip_train.set_wgrad_defer(False)

    def _post_backward(self):
        post = getattr(self.distiller, "post_backward", None)
        if post is not None:
            post()

    def _fwd(self, b: dict):
        """Zero the gradients, repack the student's weights, forward + losses."""
        packs = None
        zero = [self.flat.grads]
        if self.device.type == "cuda":
            from ..ops.backend import hip_enabled_for
            if hip_enabled_for(self.flat.data):
                from ..ops import hip_train
                # every training BN of the step gets a one-shot channel-sum region
                # of the arena; their zeroing shares the gradient-zeroing launch
                zero.append(hip_train.bn_step_begin(self.device, zero=False))
                self._bn_arena = True
                packs = self._packs
                if packs is None:
                    packs = self._packs = hip_train.PackCache()
        # the zero fills (and, for a captured step, the stem's padded image)
        # ride in the weight-pack launch
        # only the captured step's own static image may be baked into the pack
        # table: an eager step after capture (a partial batch) passing its image
        # would rebuild the table the graph still points at
        img = b.get("image")
        if not (self.use_graph and _PACK_EXTRAS and img is not None and img is self._static_img):
            img = None
        zx = zero if _PACK_EXTRAS else ()
        if packs is None or not packs.pack_all(self.device, zero=zx, image=img) or not zx:
            if len(zero) > 1 and zero[0].dtype == zero[1].dtype:
                torch._foreach_zero_(zero)
            else:
                for t in zero:
                    t.zero_()
            if packs is not None and not packs.armed:
                packs.pack_all(self.device)
        if packs is not None:
            hip_train.set_active_packs(packs)
        try:
            preds, losses = self._forward(b)
        finally:
            if packs is not None:
                packs.disarm()
                hip_train.set_active_packs(None)
        if not self.is_dot and not self._reach_ready:
            self._grad_reachability(losses)
        if self.is_dot and not self._dot_ready:
            self._dot_reachability(losses)
        return preds, losses

    def _reduce(self, replay: bool = False):
        """The step's collectives: the gradient all-reduce, then any exchange the
        distiller staged after its backward (CRD's memory-update all-gather).
        Eager between the fwd+bwd and update graphs (split mode); after a
        replay in ``events`` mode each bucket's all-reduce waits only for its
        event."""
        if self.world <= 1:
            return
        if replay and self.graph_comm == "events" and self.reducer.graph_events is not None:
            self.reducer.launch_from_events()
            self.reducer.wait_launched()
        elif self.is_dot:
            self.reducer.reduce_sets((0, 1))
        else:
            self.reducer.finish()
        exchange = getattr(self.distiller, "exchange", None)
        if exchange is not None:
            exchange()

    def _update(self, preds, target, losses):
        if self.world > 1:
            apply = getattr(self.distiller, "apply_exchange", None)
            if apply is not None:
                apply()
        self.opt.step()
        self.meters.update(preds, target, losses)

    # ------------------------------------------------------------------
    def _bn_end(self):
        if getattr(self, "_bn_arena", False):
            from ..ops import hip_train
            hip_train.bn_step_end(self.device)

    def _eager(self, b: dict):
        preds, losses = self._fwd_bwd(b, overlap_comm=True)
        self._reduce()
        self._update(preds, b["target"], losses)
        self._bn_end()
        # hand out detached outputs: a caller holding autograd-attached outputs
        # of an eager step across the hipGraph capture crashes the capture
        return preds.detach(), {k: v.detach() for k, v in losses.items()}

    def _capture(self, b: dict):
        """Capture fwd+bwd(+reduce if world==1)+update into hipGraphs.

        The warm-up step and the capture run on the SAME dedicated stream:
        MIOpen / hipBLASLt create their per-stream handles and workspaces on
        first use, which is not capturable, so that first use must happen
        eagerly on the capture stream.
        """
        static = {k: v.clone() for k, v in b.items()}
        img = self._static_img = static.get("image")
        pool = torch.cuda.graph_pool_handle()
        s = self._cap_stream = torch.cuda.Stream()
        self.reducer.avoid_streams = [s]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            # this batch's real (eager) step doubles as the capture-stream warm-up;
            # capturing records kernels without executing them
            out = self._eager(static)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if not getattr(self.distiller, "graph_capturable", True):
            # decided by the eager steps (e.g. OFD's train-mode teacher BN fell
            # back to MIOpen on some layer): stay eager for good
            self.use_graph = False
            return out
        if self.is_dot and self.dot_dual and not self.dot_single:
            try:
                return self._capture_dot_dual(static, pool, s, out)
            finally:
                self._bn_end()
        feed = None
        if self._lookahead_on(static) and getattr(self.distiller, "teacher", None) is not None:
            feed = self._capture_teacher_feed(static, pool, s)
            if self.teacher_split:
                feed.mode = "use"  # the step graph reads X; the teacher is a graph of its own
                feed.track = set()  # which X the step graph reads (only those are refreshed)
        try:
            self._capture_step(static, pool, s)
        finally:
            # the step's arena window closes with its capture: a teacher graph
            # captured next (split look-ahead) must not take regions from it,
            # or the step's zero fill at its start races that graph's replay
            self._bn_end()
            if feed is not None:
                feed.mode = None  # eager steps (e.g. a partial batch) run the teacher inline
        if feed is not None and self.teacher_split:
            self._capture_teacher_split(feed)
        return out

    def _capture_teacher_split(self, feed):
        """``RUNTIME.TEACHER_GRAPH=split``: the next batch's teacher forward as a
        single-chain graph of its own, replayed on the teacher stream beside the
        student's step graph (own memory pool: the two graphs run concurrently,
        so no block of one may be handed to the other)."""
        from ..runtime.streams import side_stream
        ts = side_stream(self.device)
        g = torch.cuda.CUDAGraph()
        ts.wait_stream(torch.cuda.current_stream())
        t_list, x_list = feed.capture_pipe(self.distiller.teacher, g, torch.cuda.graph_pool_handle(), ts,
                                           lambda: _autocast(self.device, self.dtype))
        feed.track = None
        self._tsplit = (g, t_list, x_list, ts, torch.cuda.Event(), torch.cuda.Event())
        self._tp_inflight = False
        self._x_for = None

    def _lookahead_on(self, static) -> bool:
        """Measured (profiles/r2_teacher_lookahead_ab.md): the look-ahead takes the
        CIFAR steps and the logit-only ImageNet pair down 5-30 %; with an ImageNet
        teacher whose feature maps the student also consumes (ReviewKD R34->R18)
        both sides already fill the GPU and it costs 6 %: ``auto`` skips that case."""
        if self.lookahead != "auto":
            return bool(self.lookahead)
        img = static.get("image")
        big = img is not None and img.dim() == 4 and min(img.shape[-2:]) >= 128
        needs = tuple(getattr(self.distiller, "teacher_needs", ("logits",)))
        return not (big and needs != ("logits",))

    def _capture_teacher_feed(self, static, pool, s):
        """Teacher look-ahead (``runtime/streams.py::TeacherFeed``): prime the
        persistent teacher-output buffers eagerly, capture the teacher-only
        graph that fills them for a batch that was not prefetched, and leave the
        feed in pipelined mode for the step capture that follows."""
        from ..runtime.streams import TeacherFeed
        needs = tuple(getattr(self.distiller, "teacher_needs", ()))
        feed = TeacherFeed(logits_only=needs == ("logits",))
        self._static_next = {"image": static["image"].clone()}
        feed.next_image = self._static_next["image"]
        self.distiller._teacher_feed = feed
        g_teach = torch.cuda.CUDAGraph()
        try:
            feed.mode = "teach"
            with torch.cuda.stream(s), _autocast(self.device, self.dtype):
                self.distiller.teacher_forward(None)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            # its own memory pool: replayed ahead of the step graph, its
            # temporaries (a train-mode teacher's BN regions and stats among
            # them) must not be blocks the step graph's capture reuses
            with torch.cuda.graph(g_teach, pool=torch.cuda.graph_pool_handle(), stream=s), \
                    _autocast(self.device, self.dtype):
                self.distiller.teacher_forward(None)
        except Exception:
            feed.mode = None
            self.distiller.__dict__.pop("_teacher_feed", None)
            raise
        feed.mode = "pipe"
        self._pipe = (g_teach, feed)
        self._x_for = None
        return feed

    def _capture_step(self, static, pool, s):
        g1 = torch.cuda.CUDAGraph()
        if self.world <= 1:
            with torch.cuda.graph(g1, pool=pool, stream=s):
                preds, losses = self._fwd_bwd(static, overlap_comm=False)
                self._update(preds, static["target"], losses)
            g2 = None
        else:
            with torch.cuda.graph(g1, pool=pool, stream=s):
                preds, losses = self._fwd_bwd(static, overlap_comm=self.graph_comm == "events"
                                              and "events")
            g2 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g2, pool=pool, stream=s):
                self._update(preds, static["target"], losses)
        self._bn_end()
        self._graphs = (g1, g2)
        self._static = (static, preds.detach(), {k: v.detach() for k, v in losses.items()})

    def _replay_main(self):
        """Replay the captured step graph(s) on the current stream (+ the eager
        collectives between graphs)."""
        g1, g2 = self._graphs
        g1.replay()
        if g2 is not None:
            self._reduce(replay=True)
            g2.replay()

    def _capture_dot_dual(self, static, pool, s, out):
        """DOT: the task (CE) and KD backwards are independent -- both only read
        the forward's saved tensors and write their own half of the ``[2, n]``
        gradient buffer -- so they are captured as separate graphs and replayed
        on two streams, the CE pass overlapping the KD pass (the CIFAR student's
        backward kernels are small; one pass alone leaves most CUs idle).  The CE
        graph allocates from its own memory pool and its BN scratch is tagged
        (``hip_train.set_ws_tag``), so nothing it writes aliases the KD graph.
        """
        from ..ops import hip_train
        feed = None
        needs = tuple(getattr(self.distiller, "teacher_needs", ("logits",)))
        if (self._lookahead_on(static) and needs == ("logits",)
                and getattr(self.distiller, "teacher", None) is not None):
            # look-ahead under the dual replay: the forward reads the prefetched
            # logits, and the NEXT batch's teacher runs inside the CE-backward graph
            # (beside both backward passes); the KD backward does not read them
            feed = self._capture_teacher_feed(static, pool, s)
            feed.mode = "use"
        # split: the next batch's teacher is its own graph on the teacher stream
        # (not a branch of the CE graph); the copy into X happens before the step
        in_graph = feed is not None and not self.teacher_split
        g_fwd, g_kd, g_ce, g_opt = (torch.cuda.CUDAGraph() for _ in range(4))
        with torch.cuda.graph(g_fwd, pool=pool, stream=s):
            preds, losses = self._fwd(static)
        with torch.cuda.graph(g_kd, pool=pool, stream=s):
            self.flat.bind_grads(1)
            deferred = self._arm_wgrad_defer()
            try:
                losses["loss_kd"].backward(retain_graph=True)
            finally:
                self._flush_wgrad_defer(deferred)
                join_branches()
        hip_train.set_ws_tag("dot_ce")
        try:
            with torch.cuda.stream(s):
                hip_train._ws(self.device)  # the tagged scratch exists before the capture
            with torch.cuda.graph(g_ce, pool=torch.cuda.graph_pool_handle(), stream=s):
                if in_graph:
                    with _autocast(self.device, self.dtype):
                        feed.prefetch(self.distiller.teacher)
                self.flat.bind_grads(0)
                deferred = self._arm_wgrad_defer()
                try:
                    losses["loss_ce"].backward()
                finally:
                    self._flush_wgrad_defer(deferred)
                    join_branches()
                if in_graph:
                    # join only: the KD-backward graph may still be replaying on the
                    # main stream; the copy into the teacher-output buffers it was
                    # built from happens in g_opt, after the two streams joined
                    feed.finish(copy=False)
        finally:
            hip_train.set_ws_tag(None)
            if feed is not None:
                feed.mode = None
        if self.world > 1:
            # split mode: the bucketed all-reduce runs eagerly between the backward
            # graphs (+ the post-backward hook, if any) and the optimizer graph
            if getattr(self.distiller, "post_backward", None) is not None or in_graph:
                with torch.cuda.graph(g_opt, pool=pool, stream=s):
                    if in_graph:
                        feed.commit()
                    self._post_backward()
            else:
                g_opt = None
            g_upd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_upd, pool=pool, stream=s):
                self._update(preds, static["target"], losses)
        else:
            with torch.cuda.graph(g_opt, pool=pool, stream=s):
                if in_graph:
                    feed.commit()
                self._post_backward()
                self._update(preds, static["target"], losses)
            g_upd = None
        self._bn_end()
        from ..runtime.streams import _fresh_stream, side_stream
        s2 = _fresh_stream(self.device.index or 0, (s, side_stream(self.device)))
        self._dual = (g_fwd, g_kd, g_ce, g_opt, g_upd, s2, torch.cuda.Event())
        self._graphs = (None, None)
        self._static = (static, preds.detach(), {k: v.detach() for k, v in losses.items()})
        if feed is not None and self.teacher_split:
            self._capture_teacher_split(feed)
        return out

    def _replay_dot_dual(self):
        g_fwd, g_kd, g_ce, g_opt, g_upd, s2, ev = self._dual
        cur = torch.cuda.current_stream()
        g_fwd.replay()
        ev.record(cur)
        g_kd.replay()
        s2.wait_event(ev)
        with torch.cuda.stream(s2):
            g_ce.replay()
        cur.wait_stream(s2)
        if g_opt is not None:
            g_opt.replay()
        if g_upd is not None:
            self._reduce(replay=True)
            g_upd.replay()

    def step(self, batch: dict, next_batch: dict = None):
        """Run one step; returns device ``(preds, losses)`` (no host sync).

        ``next_batch`` (optional): the batch the NEXT call will receive.  With the
        teacher look-ahead captured, its teacher forward runs during this step
        (beside the student's forward / backward / update), and the next call
        finds its teacher outputs ready.
        """
        from ..ops.hip_layers import bump_weight_generation
        bump_weight_generation()  # parameters / BN stats change: inference packs are stale
        b = self._prep(batch)
        if not self.use_graph or self.steps_done < self.warmup_eager:
            out = self._eager(b)
            self.steps_done += 1
            return out
        if self._graphs is None:
            try:
                out = self._capture(b)
            except RuntimeError as e:  # a non-capturable op: stay eager for good
                import warnings
                warnings.warn(f"hipGraph capture failed ({e}); continuing without graphs")
                self.use_graph = False
                self._graphs = self._static = self._dual = None
                self._drop_feed()
                torch.cuda.synchronize()
                out = self._eager(b)
                self.steps_done += 1
                return out
            self.steps_done += 1
            return out
        static, preds, losses = self._static
        if any(static[k].shape != v.shape for k, v in b.items()):
            # e.g. the last partial batch of an epoch: run it eagerly
            self._x_for = None
            out = self._eager(b)
            self.steps_done += 1
            return out
        if self._tsplit is not None and self._pipe is not None:
            return self._step_split(batch, b, next_batch, static, preds, losses)
        # the step's input copies in one multi-tensor launch (each separate copy is a
        # ~5 us kernel ahead of the graph)
        dst = [static[k] for k in b]
        src = [b[k] for k in b]
        if self._pipe is not None:
            g_teach, _ = self._pipe
            nxt = self._static_next["image"]
            if self._x_for is None or self._x_for is not batch.get("image"):
                torch._foreach_copy_(dst, src)
                dst, src = [], []
                nxt.copy_(static["image"], non_blocking=True)  # this batch was not prefetched
                g_teach.replay()
            if next_batch is not None and next_batch.get("image") is not None \
                    and tuple(next_batch["image"].shape) == tuple(nxt.shape):
                dst.append(nxt)
                src.append(self._prep_image(next_batch["image"]))
                self._x_for = next_batch["image"]
                self._la_misses = 0
            else:
                self._x_for = None  # the step's teacher prefetch is discarded
                self._la_misses += 1
                if self._la_misses >= 3:
                    # a caller that never passes next_batch would pay two teacher
                    # forwards per step: this step eagerly, then recapture without
                    # the look-ahead
                    self.lookahead = False
                    self.invalidate_graph()
                    out = self._eager(b)
                    self.steps_done += 1
                    return out
        if dst:
            torch._foreach_copy_(dst, src)
        if self._dual is not None:
            self._replay_dot_dual()
            self.steps_done += 1
            return preds, losses
        self._replay_main()  # (split mode: eager all-reduce between the graphs)
        self.steps_done += 1
        return preds, losses

    def _step_split(self, batch, b, next_batch, static, preds, losses):
        """A replayed step with the look-ahead teacher as its own graph: main
        stream -- wait for the teacher of this batch, ONE multi-tensor copy of
        the inputs and of its outputs T into X, the student's step graph(s);
        teacher stream -- once that copy is done, the next image into the
        teacher's input buffer and the teacher graph of the next batch."""
        g_teach, _ = self._pipe
        g_tp, t_list, x_list, ts, ev_t, ev_c = self._tsplit
        cur = torch.cuda.current_stream()
        nxt = self._static_next["image"]
        prefetched = False
        if self._tp_inflight:
            cur.wait_event(ev_t)  # T (or a discarded prefetch) is complete; nxt is free
            self._tp_inflight = False
            prefetched = self._x_for is not None and self._x_for is batch.get("image")
        dst = [static[k] for k in b]
        src = [b[k] for k in b]
        if prefetched:
            _multi_copy(dst + x_list, src + t_list)
        else:
            _multi_copy(dst, src)
            nxt.copy_(static["image"], non_blocking=True)  # this batch was not prefetched
            g_teach.replay()                                # its teacher straight into X
        nimg = None
        if next_batch is not None and next_batch.get("image") is not None \
                and tuple(next_batch["image"].shape) == tuple(nxt.shape):
            nimg = self._prep_image(next_batch["image"])
            self._x_for = next_batch["image"]
            self._la_misses = 0
        else:
            self._x_for = None
            self._la_misses += 1
            if self._la_misses >= 3:
                self.lookahead = False
                self.invalidate_graph()
                out = self._eager(b)
                self.steps_done += 1
                return out

        if nimg is not None:
            ev_c.record(cur)  # X copied (and g_teach done): T and nxt may be overwritten

        def launch_teacher():
            ts.wait_event(ev_c)
            with torch.cuda.stream(ts):
                nxt.copy_(nimg, non_blocking=True)
                g_tp.replay()
            ev_t.record(ts)
            nimg.record_stream(ts)
            self._tp_inflight = True

        if nimg is not None and self.teacher_first:
            launch_teacher()
        if self._dual is not None:
            self._replay_dot_dual()
        else:
            self._replay_main()
        if nimg is not None and not self.teacher_first:
            launch_teacher()
        self.steps_done += 1
        return preds, losses

    def invalidate_graph(self) -> None:
        """Drop captured graphs (shape change, e.g. the last partial batch)."""
        self._graphs = None
        self._static = None
        self._dual = None
        self._drop_feed()

    def _drop_feed(self) -> None:
        if self._tsplit is not None:
            if self._tp_inflight:
                torch.cuda.current_stream().wait_event(self._tsplit[4])
                self._tp_inflight = False
            torch.cuda.current_stream().synchronize()
            self._tsplit = None
        if self._pipe is not None:
            self._pipe = None
            self.distiller.__dict__.pop("_teacher_feed", None)
        self._x_for = None

    # ------------------------------------------------------------------
    def state_dict(self) -> dict:
        return self.opt.state_dict()

    def load_state_dict(self, sd: dict) -> None:
        from ..ops.hip_layers import bump_weight_generation
        bump_weight_generation()
        self.opt.load_state_dict(sd)
