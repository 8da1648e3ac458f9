"""Bucketed all-reduce of the flat gradient buffer, overlapped with backward.

Replaces ``DistributedDataParallel`` (reference `tools/train.py:86`) for the
distiller's learnable parameters only:

* only student + distiller-module gradients go on the wire (the teacher is
  frozen and never registered: 4.7 MB instead of 33 MB per step for DKD
  res32x4->res8x4);
* gradients already live in one contiguous buffer
  (:class:`..engine.optim.FlatParams`), so a bucket is a slice -- no packing
  copies -- and the collective runs on the native RCCL stream;
* buckets follow the flat layout (reverse registration order = the order
  backward produces gradients), and each bucket is launched from a
  post-accumulate-grad hook as soon as its last gradient lands, so the
  all-reduce of the head's gradients overlaps the backward of the stem;
* the 1/world averaging is NOT a separate pass: the optimizer kernel scales
  by ``grad_scale = 1/world`` while it reads the gradient anyway;
* DOT's two gradient sets are reduced (the reference's DDP syncs only the
  first backward), honouring the bf16 wire format too.

Under hipGraphs (``TrainStep``, ``DIST.GRAPH_COMM``): ``events`` (the
default at world > 1) -- the same hooks fire inside the captured backward and
record one external event per bucket where its last gradient is written;
after each replay is launched the host enqueues, on a comm stream, "wait for
bucket k's event, all-reduce bucket k" in bucket order, so the head-side
buckets are on the wire while the replay is still computing the stem's
gradients (:meth:`GradReducer.arm_capture`, :meth:`launch_from_events`).
DOT's single-pass backward writes both gradient sets of a parameter in one
launch, so each event launches both sets' slices (``sets``).  ``split``
all-reduces eagerly between the fwd+bwd and update graphs; ``capture`` puts
the collectives inside one multi-branch graph.

Bucket size: xGMI is point-to-point (7 links/GPU); RCCL's ring all-reduce of
an S-byte bucket costs ~latency + 2(N-1)/N * S / link_bw per channel, so a
few MB per bucket already amortises the ~10-20 us latency.  The overlap
comes from the buckets that complete early, so ``DIST.BUCKET_MB = 0`` (the
default) sizes them from the model: a quarter of the gradient, clamped to
[0.5, 8] MB (:func:`auto_bucket_mb`) -- four buckets for the north-star
student (4.7 MB fp32), 8 MB buckets for ImageNet students.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .dist import is_dist, get_world_size

_ARMED: list = []  # reducers currently expecting gradients


def notify_grad(*params) -> None:
    """Native backward kernels that accumulate straight into a parameter's
    flat ``.grad`` view (returning ``None`` to autograd, so no accumulate
    hook fires) report the write here, which lets the bucket holding the
    parameter launch its all-reduce as soon as it is complete."""
    if _ARMED:
        for r in list(_ARMED):
            for p in params:
                r.ready_param(p)


def auto_bucket_mb(numel: int) -> float:
    """``DIST.BUCKET_MB = 0``: a quarter of the flat fp32 gradient, clamped to
    [0.5, 8] MB.  The overlap comes from the buckets that complete early in the
    backward (the head's), so a small model wants several buckets -- the
    flagship ResNet8x4 student (4.7 MB) gets four of ~1.2 MB, the first
    launched after the last stage's backward -- while a large one keeps
    buckets big enough to amortise a collective's launch and latency over
    point-to-point xGMI (ResNet-18: 8 MB buckets)."""
    total = numel * 4 / float(1 << 20)
    return min(8.0, max(0.5, total / 4.0))


class GradReducer:
    def __init__(self, flat, bucket_mb: float = 8.0, overlap: bool = True, group=None,
                 wire_dtype: str = "fp32"):
        self.flat = flat
        self.group = group
        self.enabled = is_dist()
        self.world = get_world_size()
        self.overlap = overlap and self.enabled
        self.wire_bf16 = wire_dtype == "bf16"
        self.bytes_reduced = 0  # bytes put on the wire (tests / accounting)
        self.calls = 0
        self.early_launches = 0  # buckets launched from inside backward (overlap)
        self.avoid_streams = []  # streams the comm stream must differ from (TrainStep sets them)
        # gradient sets each bucket all-reduce covers (DOT's single-pass backward
        # writes both sets of a parameter in one launch: (0, 1)); None = the bound set
        self.sets = None
        if not bucket_mb or bucket_mb <= 0:
            bucket_mb = auto_bucket_mb(flat.numel)
        self.bucket_mb = float(bucket_mb)
        bucket_elems = max(64, int(bucket_mb * (1 << 20) / 4))
        # buckets aligned to parameter boundaries, in flat (= backward) order
        order = sorted(range(len(flat.params)), key=lambda i: flat.offsets[i])
        self.buckets = []  # list of (start, end, [param indices])
        cur, start, size = [], None, 0
        for i in order:
            o, n = flat.offsets[i], flat.params[i].numel()
            if start is None:
                start = o
            cur.append(i)
            size = o + n - start
            if size >= bucket_elems:
                self.buckets.append([start, self._end(o, n), cur])
                cur, start, size = [], None, 0
        if cur:
            self.buckets.append([start, self._end(flat.offsets[cur[-1]], flat.params[cur[-1]].numel()), cur])
        if self.buckets:
            self.buckets[-1][1] = flat.numel  # include tail padding
        self._param_bucket = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self._param_bucket[i] = b
        self._index = {id(p): i for i, p in enumerate(flat.params)}
        # gradient contributions per parameter and step, learned on the first
        # armed step (a "calibration" backward that launches nothing early):
        # autograd's accumulate hook and the native kernels that write straight
        # into the flat buffer (notify_grad) both count
        self._expected = None
        self._calib = None
        self._pending = []
        self._next = 0
        self._works = {}
        self._wires = {}
        self._hooks = []
        self._armed = False
        self._error = None
        # captured-backward overlap (DIST.GRAPH_COMM=events, see arm_capture)
        self._arm_stream = None    # the stream the armed backward started on
        self._from_events = False  # launching behind graph events (no stream joins)
        self._cap = None           # events recorded so far while capturing: [(bucket, event)]
        self._cap_flush = None     # called before a bucket's event is recorded
        self.graph_events = None   # [(bucket, event)] of the captured graph, bucket order
        self._comm = None
        if self.overlap:
            for i, p in enumerate(flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    @staticmethod
    def _end(o, n):
        from ..engine.optim import ALIGN
        return o + ((n + ALIGN - 1) // ALIGN) * ALIGN

    # ------------------------------------------------------------------
    def _make_hook(self, i):
        def hook(_p):
            if self._armed:
                self._ready(i)
        return hook

    def _ready(self, i):
        if self._calib is not None:
            self._calib[i] += 1
            return
        b = self._param_bucket[i]
        self._pending[b] -= 1
        if self._pending[b] < 0 and b < self._next and self._error is None:
            # more contributions than the calibration step counted, after the
            # bucket was already all-reduced: the reduced values are stale.
            # Recorded, not raised here: the peers are about to enter the
            # remaining buckets' collectives, so finish() drains them first
            self._error = (
                f"GradReducer: parameter {i} received a gradient contribution after its "
                f"bucket {b} was launched (calibrated {self._expected[i] if self._expected else '?'} "
                "contributions); disable DIST.OVERLAP or keep the backward graph static")
        # strictly in bucket order: every rank issues the same collective
        # sequence even if two buckets complete in a different order
        while self._next < len(self.buckets) and self._pending[self._next] <= 0:
            if self._cap is not None:
                self._signal(self._next)
            else:
                self._launch(self._next, async_op=True)
                self.early_launches += 1
            self._next += 1

    def ready_param(self, p) -> None:
        i = self._index.get(id(p))
        if i is not None and self._armed:
            self._ready(i)

    def _slice(self, b):
        s, e, _ = self.buckets[b]
        return self.flat.grads[self.flat._bound][s:e]

    def _wire_buf(self, key, n, device):
        """Persistent bf16 wire buffer (allocated once, reused every step)."""
        w = self._wires.get(key)
        if w is None or w.numel() != n or w.device != device:
            w = self._wires[key] = torch.empty(n, dtype=torch.bfloat16, device=device)
        return w

    def _join_writers(self, stream) -> None:
        """Make ``stream`` wait for every stream a gradient of the step may be
        written on: the one the backward started on (``arm``) and the residual
        branch streams.  A bucket completes in the hook of its LAST gradient,
        which runs with that gradient's stream current -- a projection
        shortcut's weight gradient is written on the branch stream, the rest
        of its bucket on the main one (an all-reduce ordered after the branch
        alone raced the main stream's writes: replicas diverged ~1 run in 3)."""
        from ..runtime import streams as S
        dev = torch.cuda.current_device()
        capturing = self._cap is not None
        for o in (self._arm_stream, S._branch_streams.get(dev)):
            if o is None or o.cuda_stream == stream.cuda_stream:
                continue
            if capturing:
                # inside a capture only a stream that is part of it can be
                # joined (a branch stream the captured step never forked is idle)
                with torch.cuda.stream(o):
                    if not torch.cuda.is_current_stream_capturing():
                        continue
            stream.wait_stream(o)

    def _launch(self, b, async_op):
        if self._arm_stream is not None and self._cap is None and not self._from_events:
            self._join_writers(torch.cuda.current_stream())
        if self.sets is not None:  # every listed gradient set's slice of the bucket
            s, e, _ = self.buckets[b]
            for k in self.sets:
                self._launch_t((b, k), self.flat.grads[k][s:e], async_op)
            return
        self._launch_t(b, self._slice(b), async_op)

    def _launch_t(self, key, t, async_op):
        self.bytes_reduced += t.numel() * (2 if self.wire_bf16 else 4)
        self.calls += 1
        if self.wire_bf16:
            tb = self._wire_buf(("b", key), t.numel(), t.device)
            tb.copy_(t)
            work = dist.all_reduce(tb, group=self.group, async_op=True)
            self._works[key] = (work, t, tb)
        else:
            work = dist.all_reduce(t, group=self.group, async_op=async_op)
            self._works[key] = (work, None, None)

    def arm(self) -> None:
        """Call before a backward whose gradients should be reduced on the fly."""
        if not self.enabled:
            return
        self._works = {}
        self._next = 0
        self._armed = self.overlap
        if not self._armed:
            return
        self._arm_stream = torch.cuda.current_stream() if self.flat.grads.is_cuda else None
        if self._expected is None:
            self._calib = [0] * len(self.flat.params)
        else:
            self._pending = [sum(self._expected[i] for i in idx) for (_, _, idx) in self.buckets]
        _ARMED.append(self)

    def finish(self) -> None:
        """Launch any bucket not yet launched and wait for all of them."""
        if not self.enabled:
            return
        if self._calib is not None:
            self._expected, self._calib = self._calib, None
        elif self._armed and any(p < 0 for p in self._pending) and self._error is None:
            self._error = (f"GradReducer: bucket contribution counts went negative "
                           f"{self._pending} (a parameter got more gradient writes than "
                           f"the calibration step counted)")
        launched = {k[0] if isinstance(k, tuple) else k for k in self._works}
        for b in range(len(self.buckets)):
            if b not in launched:
                self._launch(b, async_op=True)
        for b, (work, t, tb) in self._works.items():
            if work is not None:
                work.wait()
            if tb is not None:
                t.copy_(tb)
        self._works = {}
        self._armed = False
        if self in _ARMED:
            _ARMED.remove(self)
        # every bucket was launched and drained before raising, so no peer is
        # left waiting in a collective this rank skipped (a peer that goes on
        # to the next step fails on the process group's timeout, not a hang)
        err, self._error = self._error, None
        if err is not None:
            raise RuntimeError(err)

    # ------------------------------------------------------------------
    # Overlap under hipGraphs (DIST.GRAPH_COMM=events).  RCCL collectives
    # captured INSIDE the step graph make it a multi-branch graph, which ROCm's
    # executor runs slowly (scripts/launch_floor_probe.py); instead the captured
    # backward records one external event per bucket at the point where the
    # bucket's last gradient is written, and after launching the replay the
    # host enqueues, on a comm stream, "wait for bucket k's event, all-reduce
    # bucket k" for every bucket in order: the all-reduce of the head's
    # buckets runs while the replay is still computing the stem's gradients.
    def arm_capture(self, flush=None) -> None:
        """Call inside the capture, before the backward.  ``flush`` (optional)
        runs before each bucket's event is recorded (the deferred weight-gradient
        reductions: their layers' gradients are only final after it)."""
        if not self.enabled or self._expected is None:
            raise RuntimeError("GradReducer.arm_capture: needs a calibrated eager step first")
        self._works = {}
        self._next = 0
        self._armed = True
        self._cap = []
        self._cap_flush = flush
        # the capturing stream: a bucket can complete inside a hook that the
        # autograd engine runs with ANOTHER current stream (a leaf's
        # AccumulateGrad runs on the stream the leaf was made on, not capturing)
        self._cap_stream = torch.cuda.current_stream()
        self._arm_stream = self._cap_stream
        self._pending = [sum(self._expected[i] for i in idx) for (_, _, idx) in self.buckets]
        _ARMED.append(self)

    def _signal(self, b) -> None:
        if self._cap_flush is not None:
            # on the CAPTURING stream: the hook that completes a bucket may run
            # with another current stream (a leaf's AccumulateGrad), and a flush
            # enqueued there would run once, eagerly, instead of in every replay
            with torch.cuda.stream(self._cap_stream):
                self._cap_flush()
        from ..runtime.streams import HipEvent
        # the event must also cover gradients written on a residual branch
        # stream (a join edge in the captured graph; see _join_writers)
        self._join_writers(self._cap_stream)
        ev = HipEvent()  # (torch.cuda.Event(external=True) is refused on ROCm)
        ev.record(external=True, stream=self._cap_stream)
        self._cap.append((b, ev))

    def abort_capture(self) -> None:
        """A capture failed mid-backward: leave the capture mode (the eager
        fallback step must launch its buckets normally)."""
        self._cap = None
        self._cap_flush = None
        self._armed = False
        self.graph_events = None
        if self in _ARMED:
            _ARMED.remove(self)

    def finish_capture(self) -> None:
        """End of the captured backward: events for the buckets not signalled
        yet (all their gradients are written by now)."""
        try:
            if any(p < 0 for p in self._pending):
                raise RuntimeError(f"GradReducer: bucket contribution counts went negative "
                                   f"{self._pending} in the captured backward")
            while self._next < len(self.buckets):
                self._signal(self._next)
                self._next += 1
            self.graph_events = list(self._cap)
        finally:
            self._cap = None
            self._cap_flush = None
            self._armed = False
            if self in _ARMED:
                _ARMED.remove(self)

    def launch_from_events(self) -> None:
        """After the replay of a graph captured with :meth:`arm_capture`: every
        bucket's all-reduce on the comm stream, each behind its event; the
        caller then runs :meth:`wait_launched` before the optimizer."""
        if self._comm is None:
            from ..runtime import streams as S
            idx = torch.cuda.current_device()
            # never one of the step's other live streams (teacher, branch,
            # wgrad, capture): the bucket all-reduces would queue behind them
            avoid = [S._streams.get(idx), S._branch_streams.get(idx)] + list(self.avoid_streams)
            # high priority: a bucket's wait + all-reduce never queues behind the
            # teacher's or the student's kernels on a shared hardware queue
            # (docs/DESIGN.md 4, stream -> queue map)
            self._comm = S._fresh_stream(idx, avoid, priority=-1)
        # (no wait on the current stream: that would wait for the whole replay;
        # each all-reduce waits only for its bucket's event)
        self._works = {}
        self._from_events = True  # each bucket's event already covers its writers
        try:
            with torch.cuda.stream(self._comm):
                for b, ev in self.graph_events:
                    ev.wait(self._comm)
                    self._launch(b, async_op=True)
                    self.early_launches += 1
        finally:
            self._from_events = False

    def wait_launched(self) -> None:
        cur = torch.cuda.current_stream()
        if self._comm is not None:
            cur.wait_stream(self._comm)  # the wire copies / waits enqueued there
        for b, (work, t, tb) in self._works.items():
            if work is not None:
                work.wait()  # the current stream waits for the collective
            if tb is not None:
                t.copy_(tb)
        self._works = {}

    def calibrate(self) -> None:
        """Count each parameter's gradient contributions in the backward that
        follows, launching nothing (a trainer that reduces whole gradient sets
        itself, DOT, still needs the counts for :meth:`arm_capture`); close
        with :meth:`end_calibration`."""
        if not self.enabled or self._expected is not None:
            return
        self._works = {}
        self._next = 0
        self._armed = True
        self._calib = [0] * len(self.flat.params)
        _ARMED.append(self)

    def end_calibration(self) -> None:
        if self._calib is not None:
            self._expected, self._calib = self._calib, None
        self._armed = False
        if self in _ARMED:
            _ARMED.remove(self)

    def reduce_all(self) -> None:
        """Non-overlapped reduction of the currently bound gradient set."""
        if not self.enabled:
            return
        self._armed = False
        self._works = {}
        self.finish()

    def reduce_sets(self, sets=(0,)) -> None:
        """Reduce whole gradient sets (DOT: both halves of the [2, n] buffer in one call)."""
        if not self.enabled:
            return
        g = self.flat.grads
        if len(sets) == g.shape[0]:
            t = g.view(-1)
        else:
            t = g[sets[0]]
        self.bytes_reduced += t.numel() * (2 if self.wire_bf16 else 4)
        self.calls += 1
        if self.wire_bf16:
            tb = self._wire_buf(("sets", tuple(sets)), t.numel(), t.device)
            tb.copy_(t)
            dist.all_reduce(tb, group=self.group)
            t.copy_(tb)
        else:
            dist.all_reduce(t, group=self.group)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
