"""Attention Transfer, Zagoruyko & Komodakis 2017 (reference `distillers/AT.py:8-50`).

Per stage: ``a(f) = normalize(mean_c f^p)`` over the flattened spatial map,
loss = ``mean((a(f_s) - a(f_t))^2)`` summed over stages 1..N.  On MI355X the
per-stage loss is one fused HIP kernel (channel reduction + L2 normalise +
squared difference, fwd and bwd) -- :func:`..ops.feat_losses.at_loss`.
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class AT(Distiller):
    teacher_needs = ("feats",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.p = cfg.AT.P
        self.ce_loss_weight = cfg.AT.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.AT.LOSS.FEAT_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_feat = self.feat_loss_weight * FL.at_loss(
            feature_student["feats"][1:], feature_teacher["feats"][1:], self.p)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
