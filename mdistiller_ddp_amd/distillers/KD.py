"""Vanilla KD, Hinton et al. 2015 (reference `distillers/KD.py:16-39`).

``loss_ce = CE_W * CE(s, y)``; ``loss_kd = KD_W * T^2 * KL(softmax(t/T) || softmax(s/T))``
(summed over classes, mean over batch).  Both come from one fused HIP launch
on MI355X (:func:`..ops.losses.ce_kd`).
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L


class KD(Distiller):
    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.request_logits_only()
        self.temperature = cfg.KD.TEMPERATURE
        self.ce_loss_weight = cfg.KD.LOSS.CE_WEIGHT
        self.kd_loss_weight = cfg.KD.LOSS.KD_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, _ = self.student(image)
        logits_teacher, _ = t_out.get()
        loss_ce, loss_kd = L.ce_kd(logits_student, logits_teacher, target, self.temperature,
                                   self.ce_loss_weight, self.kd_loss_weight)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_kd}
