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

import threading

import torch

_state = {"enabled": True}
_streams: dict = {}
_lock = threading.Lock()


def set_enabled(flag: bool) -> None:
    _state["enabled"] = bool(flag)


def enabled() -> bool:
    return _state["enabled"]


def side_stream(device) -> "torch.cuda.Stream":
    idx = torch.device(device).index or 0
    with _lock:
        s = _streams.get(idx)
        if s is None:
            s = torch.cuda.Stream(device=idx)
            _streams[idx] = s
        return s


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
