"""Similarity-Preserving KD, ICCV 2019 (reference `distillers/SP.py:8-49`).

Row-normalised B x B Gram matrices of the last stage's features; squared
Frobenius difference / B^2.  The Grams are MFMA GEMMs (B x CHW x B).
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class SP(Distiller):
    teacher_needs = ("feats",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.SP.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.SP.LOSS.FEAT_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_feat = self.feat_loss_weight * FL.sp_loss(
            [feature_student["feats"][-1]], [feature_teacher["feats"][-1]])
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat.reshape(())}
