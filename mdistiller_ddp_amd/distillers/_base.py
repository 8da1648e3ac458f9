"""Distiller base classes (reference `mdistiller/distillers/_base.py:6-66`).

A distiller owns a trainable ``student`` and a frozen ``teacher``:

* ``train()`` keeps the teacher in eval mode (BN running stats frozen);
* ``forward(image=..., target=..., epoch=...)`` returns
  ``(student_logits, {"loss_ce": ..., "loss_kd": ...})`` in training mode and
  the student logits in eval mode;
* ``get_learnable_parameters()`` = student parameters + the distiller's own
  modules (connectors, regressors, embeddings);
* ``get_extra_parameters()`` = number of parameters the method adds.

MI355X-native differences (not visible in the API):

* the teacher is frozen at construction (``requires_grad=False``), so the
  data-parallel layer never ships its gradients (the reference all-reduces
  33 MB per step instead of 4.7 MB);
* :meth:`teacher_forward` runs the teacher under ``no_grad`` on the
  runtime's teacher stream (:mod:`..runtime.streams`), so it overlaps the
  student forward instead of running after it;
* ``epoch`` may be a Python number or a 0-d device tensor; warm-up factors
  are computed with tensor ops in the latter case so a captured hipGraph can
  replay the step with a changing epoch.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import losses as L
from ..runtime import streams


def warmup_factor(epoch, warmup):
    """``min(epoch / warmup, 1)`` for a float or a device-tensor epoch."""
    if warmup is None or warmup <= 0:
        return 1.0
    if isinstance(epoch, torch.Tensor):
        return torch.clamp(epoch.float() / float(warmup), max=1.0)
    return min(float(epoch) / float(warmup), 1.0)


class Distiller(nn.Module):
    #: which teacher outputs the method consumes ("logits", "feats", "preact")
    teacher_needs = ("logits",)
    #: False when the training step contains host-synchronising ops (KDSVD's
    #: batched SVD) and therefore cannot be captured into a hipGraph
    graph_capturable = True

    def __init__(self, student: nn.Module, teacher: nn.Module):
        super().__init__()
        self.student = student
        self.teacher = teacher
        for p in self.teacher.parameters():
            p.requires_grad_(False)
        self._teacher_train_bn = False

    @property
    def module(self):
        return self

    def train(self, mode: bool = True):
        if not isinstance(mode, bool):
            raise ValueError("training mode is expected to be boolean")
        self.training = mode
        for m in self.children():
            m.train(mode)
        self.teacher.train(mode and self._teacher_train_bn)
        return self

    def request_logits_only(self) -> None:
        """Logit-only methods: models skip storing pre-activation features."""
        for m in (self.student, self.teacher):
            if hasattr(m, "request_features"):
                m.request_features(False)

    # parameters ------------------------------------------------------------
    def distill_modules(self):
        """Sub-modules (besides student/teacher) holding trainable params."""
        return [m for n, m in self.named_children() if n not in ("student", "teacher")]

    def get_learnable_parameters(self):
        params = [p for p in self.student.parameters()]
        for m in self.distill_modules():
            params += [p for p in m.parameters() if p.requires_grad]
        return params

    def get_extra_parameters(self) -> int:
        return sum(p.numel() for m in self.distill_modules() for p in m.parameters())

    # forward ---------------------------------------------------------------
    def teacher_forward(self, image):
        """Frozen teacher forward issued on the teacher stream.

        Returns a :class:`~..runtime.streams.TeacherOutput`; call ``.get()``
        after issuing the student forward so the two overlap on the GPU.
        """
        # OFD keeps the teacher's BN in training mode: on the GPU its
        # layers run as native conv + batch-statistics BN (ops/hip_train.py::
        # conv_trainbn_nograd), which is capture-safe -- MIOpen's bf16 train-mode
        # BN replayed from a hipGraph went non-finite run to run (r1 evidence,
        # profiles/r1_ofd_graph_ab.md)
        feed = self.__dict__.get("_teacher_feed")
        if feed is not None:  # TrainStep's teacher look-ahead (runtime/streams.py::TeacherFeed)
            return feed.forward(self.teacher, image)
        return streams.run_teacher_async(self.teacher, image)

    def forward_train(self, **kwargs):
        raise NotImplementedError

    def forward_test(self, image):
        return self.student(image)[0]

    def forward(self, **kwargs):
        if self.training:
            return self.forward_train(**kwargs)
        return self.forward_test(kwargs["image"])


class Vanilla(nn.Module):
    """Plain CE training of the student (`_base.py:47-66`); key ``"ce"``."""

    def __init__(self, student: nn.Module):
        super().__init__()
        self.student = student
        # CE on the logits only: no pre-activation features are stored, so every
        # native BN backward takes its sums from the consumer's dgrad (BnLink)
        if hasattr(student, "request_features"):
            student.request_features(False)

    @property
    def module(self):
        return self

    def get_learnable_parameters(self):
        return [p for p in self.student.parameters()]

    def get_extra_parameters(self) -> int:
        return 0

    def forward_train(self, image, target, **kwargs):
        logits, _ = self.student(image)
        return logits, {"ce": L.ce(logits, target)}

    def forward_test(self, image):
        return self.student(image)[0]

    def forward(self, **kwargs):
        if self.training:
            return self.forward_train(**kwargs)
        return self.forward_test(kwargs["image"])
