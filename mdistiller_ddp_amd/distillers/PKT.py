"""Probabilistic Knowledge Transfer (reference `distillers/PKT.py:8-63`).

Cosine-similarity matrices of the pooled features (B x B), shifted to [0, 1],
row-normalised into conditional probabilities, KL(teacher || student).
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class PKT(Distiller):
    teacher_needs = ("pooled",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.PKT.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.PKT.LOSS.FEAT_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_feat = self.feat_loss_weight * FL.pkt_loss(
            feature_student["pooled_feat"], feature_teacher["pooled_feat"])
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
