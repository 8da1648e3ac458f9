"""Decoupled Knowledge Distillation, CVPR 2022 (reference `distillers/DKD.py:8-84`).

``loss_kd = min(epoch / WARMUP, 1) * (ALPHA * TCKD + BETA * NCKD) * T^2 / B`` where
TCKD is the KL between the binary (target, non-target) distributions and
NCKD the KL between the softmaxes over the non-target classes.  The fused HIP
kernel excludes the target column explicitly (the reference subtracts
``1000 * gt_mask`` from the tempered logits, which is the same in fp32 and
fragile in bf16), computing everything in fp32.
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L


class DKD(Distiller):
    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.request_logits_only()
        self.ce_loss_weight = cfg.DKD.CE_WEIGHT
        self.alpha = cfg.DKD.ALPHA
        self.beta = cfg.DKD.BETA
        self.temperature = cfg.DKD.T
        self.warmup = cfg.DKD.WARMUP

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, _ = self.student(image)
        logits_teacher, _ = t_out.get()
        loss_ce, loss_dkd = L.ce_dkd(logits_student, logits_teacher, target, self.ce_loss_weight,
                                     self.alpha, self.beta, self.temperature,
                                     epoch=kwargs.get("epoch"), warmup=self.warmup)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_dkd}
