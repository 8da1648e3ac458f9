"""Teacher/student stream overlap.

The teacher is a frozen, no-grad network that depends only on the input
batch, so its forward is issued first on a dedicated HIP stream and the
student forward is issued on the current stream right after it; the two run
concurrently on the GPU (different CUs), and the loss waits on an event.
This is the "teacher and student forward passes overlap on separate HIP
streams" item of the design (the reference runs them back to back on one
stream, `distillers/KD.py:26-28`).

Works under ``torch.cuda.graph`` capture too: the side stream forks from and
joins back into the capturing stream through events, which hipGraph records
as a fork/join in the graph.
"""
from __future__ import annotations

import os
import threading

import torch

_state = {"enabled": True}
_streams: dict = {}
_lock = threading.Lock()


class HipEvent:
    """A raw HIP event whose record inside a stream capture becomes an
    EXTERNAL event-record node of the graph (csrc/events.hip): a stream
    outside the graph can wait on it after the replay has been launched.
    (PyTorch's ROCm build refuses ``torch.cuda.Event(external=True)``.)"""

    def __init__(self):
        import ctypes
        from ..ops import _ext
        h = ctypes.c_void_p(0)
        _ext.call("mda_event_create", h)
        self.handle = h.value

    # how an external record / wait is put into a capture: 2 = an explicit
    # event node added to the capturing graph (csrc/events.hip), 1 = the
    # hipEventRecordExternal / hipEventWaitExternal flags
    MODE = 2

    def record(self, external: bool = True, stream=None) -> None:
        from ..ops import _ext
        _ext.call("mda_event_record", self.handle, self.MODE if external else 0,
                  stream=None if stream is None else stream.cuda_stream)

    def wait(self, stream=None, external: bool = False) -> None:
        """Make ``stream`` (default: the current one) wait for the last record
        (``external``: as a wait node of the graph the stream is capturing)."""
        from ..ops import _ext
        _ext.call("mda_stream_wait_event", self.handle, self.MODE if external else 0,
                  stream=None if stream is None else stream.cuda_stream)

    def __del__(self):
        try:
            from ..ops import _ext
            if self.handle:
                _ext.call("mda_event_destroy", self.handle)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def set_enabled(flag: bool) -> None:
    _state["enabled"] = bool(flag)


def enabled() -> bool:
    return _state["enabled"]


def _fresh_stream(idx, avoid=(), priority: int = 0) -> "torch.cuda.Stream":
    """A pool stream that is not the current stream nor any in ``avoid``.

    ``torch.cuda.Stream()`` hands out the device's pool streams round-robin
    (32 per priority): after enough TrainSteps (capture, DOT-dual, branch and
    teacher streams) a new draw can alias a stream already in use, so draw
    again until it differs (the pool has more streams than a step uses)."""
    bad = {torch.cuda.current_stream(idx).cuda_stream}
    bad.update(a.cuda_stream for a in avoid if a is not None)
    s = torch.cuda.Stream(device=idx, priority=priority)
    for _ in range(64):
        if s.cuda_stream not in bad:
            break
        s = torch.cuda.Stream(device=idx, priority=priority)
    return s


def side_stream(device) -> "torch.cuda.Stream":
    idx = torch.device(device).index or 0
    with _lock:
        s = _streams.get(idx)
        if s is None:
            # (a CU-masked or prioritised teacher queue was measured slower or
            # no better, profiles/r6_ab.md "Teacher placement")
            s = _fresh_stream(idx, (_branch_streams.get(idx),))
            _streams[idx] = s
        return s


def renew(device) -> None:
    """Forget this device's cached teacher and branch streams: the next use
    takes fresh ones from the stream pool.  Called when a training step is
    built, so every step gets its streams in the same relative order as in a
    fresh process.  (HIP assigns a stream's hardware queue at creation; with
    the 4 queues of a process, which of a step's concurrently replayed streams
    share a queue decides whether they overlap -- DOT's dual-stream step ran
    1.33 ms/step alone and 1.59-1.60 after another DOT or two other configs
    in the same process, `profiles/r3_dot_history.md`.)  The pool is
    round-robin, so a "fresh" draw can wrap around onto a live stream:
    :func:`_fresh_stream` skips the current one, and the launch helpers run
    inline when the side stream still equals the current stream."""
    idx = torch.device(device).index or 0
    with _lock:
        _streams.pop(idx, None)
        _branch_streams.pop(idx, None)


def _tensors(obj, out):
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _tensors(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _tensors(o, out)
    return out


class TeacherOutput:
    """Outputs produced on the teacher stream; ``get()`` joins the streams."""

    def __init__(self, value, event=None, stream=None):
        self._value = value
        self._event = event
        self._joined = event is None

    def get(self):
        if not self._joined:
            cur = torch.cuda.current_stream()
            cur.wait_event(self._event)
            for t in _tensors(self._value, []):
                t.record_stream(cur)
            self._joined = True
        return self._value


def run_teacher_async(teacher, image, train_bn: bool = False) -> TeacherOutput:
    if not (image.is_cuda and _state["enabled"]):
        with torch.no_grad():
            return TeacherOutput(teacher(image))
    s = side_stream(image.device)
    cur = torch.cuda.current_stream()
    if s.cuda_stream == cur.cuda_stream:
        # an aliased pool stream: a fork onto the same stream is no fork
        with torch.no_grad():
            return TeacherOutput(teacher(image))
    s.wait_stream(cur)
    with torch.cuda.stream(s), torch.no_grad():
        image.record_stream(s)
        out = teacher(image)
        ev = torch.cuda.Event()
        ev.record(s)
    return TeacherOutput(out, ev, s)


def run_teacher(teacher, image, train_bn: bool = False):
    """Synchronous convenience wrapper (joins immediately)."""
    return run_teacher_async(teacher, image, train_bn).get()


class _TrackDict(dict):
    """A teacher-output dict that records which entries are read
    (TeacherFeed.track): reading a key marks EVERY tensor under it (a list
    handed on may be consumed by C++ code -- torch.cat, zip -- that no Python
    hook sees, so the granularity stays the key: FitNet reads "feats", not
    "preact_feats")."""

    def __init__(self, items, used):
        super().__init__(items)
        self._used = used

    def _mark(self, v):
        for t in _tensors(v, []):
            self._used.add(id(t))
        return v

    def __getitem__(self, k):
        return self._mark(super().__getitem__(k))

    def get(self, k, default=None):
        return self._mark(super().get(k, default))

    def values(self):
        return [self._mark(v) for v in super().values()]

    def items(self):
        return [(k, self._mark(v)) for k, v in super().items()]

    def __iter__(self):
        return iter(list(self.keys()))


def _track_struct(obj, used):
    """Wrap the dicts of a teacher-output structure; every tensor outside a
    dict (the logits) counts as read."""
    if isinstance(obj, torch.Tensor):
        used.add(id(obj))
        return obj
    if isinstance(obj, (list, tuple)):
        return type(obj)(_track_struct(o, used) for o in obj)
    if isinstance(obj, dict):
        return _TrackDict(obj, used)
    return obj


def _clone_struct(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().clone(memory_format=torch.preserve_format)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_clone_struct(o) for o in obj)
    if isinstance(obj, dict):
        return {k: _clone_struct(v) for k, v in obj.items()}
    return obj


def _copy_struct(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src)
    elif isinstance(dst, (list, tuple)):
        for d, s_ in zip(dst, src):
            _copy_struct(d, s_)
    elif isinstance(dst, dict):
        for k, d in dst.items():
            _copy_struct(d, src[k])


class TeacherFeed:
    """Teacher look-ahead: a software pipeline across training steps.

    The teacher is frozen, so its forward for batch t+1 does not depend on the
    student update of step t.  A captured step (``engine/step.py``) therefore
    runs the student's forward / backward / update of batch t on the current
    stream while the teacher forward of batch t+1 runs on the teacher stream,
    and at the end of the step moves that result into the persistent buffers
    ``X`` the next step's loss reads.  Every step still runs exactly one
    teacher forward (of fresh data) and one student step; the critical path
    becomes max(teacher, student) instead of teacher + student backward.

    Modes: ``None`` -- inline (teacher of the current batch, joined before
    the loss); ``"teach"`` -- teacher of :attr:`next_image` straight into
    ``X`` (priming); ``"pipe"`` -- hand out ``X`` and launch the teacher of
    :attr:`next_image` (joined and copied into ``X`` by :meth:`finish`).
    ``logits_only`` keeps just the logits (KD-style methods ignore the
    teacher's features, so those are not copied).
    """

    def __init__(self, logits_only: bool = False):
        self.mode = None
        self.next_image = None
        self.X = None
        self.logits_only = logits_only
        self._pending = None
        # while a set: ids of the X tensors the consumer reads (the split
        # teacher graph's per-step X <- T copy then skips the others: FitNet
        # reads one teacher feature map of the ten the teacher returns)
        self.track = None

    def _keep(self, out):
        if self.logits_only and isinstance(out, (list, tuple)) and len(out) == 2:
            return (out[0], None)
        return out

    def forward(self, teacher, image):
        if self.mode == "teach":
            out = self._keep(run_teacher_async(teacher, self.next_image).get())
            if self.X is None:
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("TeacherFeed: prime the buffers eagerly before capture")
                self.X = _clone_struct(out)
            else:
                _copy_struct(self.X, out)
            return TeacherOutput(self.X)
        if self.mode in ("pipe", "use"):
            if self.X is None:
                raise RuntimeError("TeacherFeed: pipelined step before the buffers were primed")
            if self.mode == "pipe":
                self.prefetch(teacher)
            if self.track is not None:
                return TeacherOutput(_track_struct(self.X, self.track))
            return TeacherOutput(self.X)
        return run_teacher_async(teacher, image)

    def prefetch(self, teacher) -> None:
        """Launch the teacher forward of :attr:`next_image` on the teacher stream
        (``"use"`` mode leaves this to the caller, e.g. DOT's CE-backward graph)."""
        self._pending = run_teacher_async(teacher, self.next_image)

    def finish(self, copy: bool = True) -> None:
        """End of a pipelined step: join the prefetch and move it into ``X``.

        ``copy=False`` only joins the teacher stream and keeps the result for a
        later :meth:`commit` -- for a caller whose other work may still read
        ``X`` concurrently (DOT's KD-backward graph replays beside the CE
        graph that hosts the prefetch; the copy goes after their join)."""
        if self._pending is not None:
            out = self._keep(self._pending.get())
            self._pending = None
            if copy:
                _copy_struct(self.X, out)
            else:
                self._joined = out

    def capture_pipe(self, teacher, graph, pool, stream, autocast):
        """Capture the teacher forward of :attr:`next_image` as its OWN
        single-chain graph on ``stream`` (``RUNTIME.TEACHER_GRAPH=split``).

        Its outputs ``T`` live in the graph's private pool; the training step
        copies them into ``X`` (the buffers the student graph reads) at the
        start of the next step, in the same launch as its input copies.  A
        graph with two parallel branches costs ROCm's executor ~2.5 us per
        kernel and serialised the branches in this process
        (``scripts/launch_floor_probe.py``); two single-chain graphs on two
        streams are two hardware queues.  Returns the flat (T, X) lists."""
        with torch.cuda.stream(stream), torch.no_grad(), autocast():
            self._keep(teacher(self.next_image))  # warm-up on the stream (handles, caches)
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, pool=pool, stream=stream), torch.no_grad(), autocast():
            T = self._keep(teacher(self.next_image))
        t_list, x_list = _tensors(T, []), _tensors(self.X, [])
        if len(t_list) != len(x_list) or any(a.shape != b.shape for a, b in zip(t_list, x_list)):
            raise RuntimeError("TeacherFeed: pipelined teacher outputs do not match the primed buffers")
        if self.track:
            keep = [k for k, x in enumerate(x_list) if id(x) in self.track]
            t_list, x_list = [t_list[k] for k in keep], [x_list[k] for k in keep]
        return t_list, x_list

    def commit(self) -> None:
        """Copy a result joined by ``finish(copy=False)`` into ``X``."""
        out = getattr(self, "_joined", None)
        if out is not None:
            _copy_struct(self.X, out)
            self._joined = None


# ---------------------------------------------------------------------------
# Intra-block branch concurrency (round 3).  A residual block's projection
# shortcut (1x1 conv + BN) is independent of its main path until the
# residual add, so the student issues it on a BRANCH stream forked from the
# current one: the forward shortcut runs beside conv1 / conv2, and autograd
# runs its backward (BN backward, dgrad, wgrad) on the same branch stream,
# beside the main path's dgrad chain.  Native backward kernels write some
# gradients straight into the flat buffer (no autograd edge back to the
# caller), so whoever runs the backward joins every branch stream used
# (``join_branches``) before reading the gradients; hipGraph records the
# fork/join as parallel branches of the captured step.
# Off by default: measured slower on every CIFAR student (profiles/r3_branch_fork_ab.md):
# the captured cross-stream edges cost more than the shortcut overlap saves.
_branch = {"enabled": os.environ.get("MDA_BRANCH_STREAMS", "0") == "1", "used": set()}
_branch_streams: dict = {}


def set_branches(flag: bool) -> None:
    _branch["enabled"] = bool(flag)


def branches_enabled() -> bool:
    return _branch["enabled"]


def branch_stream(device) -> "torch.cuda.Stream":
    idx = torch.device(device).index or 0
    with _lock:
        s = _branch_streams.get(idx)
        if s is None:
            s = _fresh_stream(idx, (_streams.get(idx),))
            _branch_streams[idx] = s
        return s


def run_branch(x: torch.Tensor, fn):
    """``fn(x)`` on the branch stream (training forward on a GPU), joined back
    into the current stream before the result is returned; otherwise inline."""
    if not (_branch["enabled"] and x.is_cuda and torch.is_grad_enabled()):
        return fn(x)
    cur = torch.cuda.current_stream(x.device)
    s = branch_stream(x.device)
    if s.cuda_stream == cur.cuda_stream:
        return fn(x)
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        out = fn(x)
    x.record_stream(s)
    cur.wait_stream(s)
    for t in _tensors(out, []):
        t.record_stream(cur)
    _branch["used"].add(x.device.index or 0)
    return out


def join_branches() -> None:
    """Make the current stream wait for every branch stream used (gradients
    the branch's native backward wrote directly)."""
    if not _branch["used"]:
        return
    cur = torch.cuda.current_stream()
    for idx in list(_branch["used"]):
        s = _branch_streams.get(idx)
        if s is not None and s.cuda_stream != cur.cuda_stream:
            cur.wait_stream(s)
