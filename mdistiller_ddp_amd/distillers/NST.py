"""Neuron Selectivity Transfer (reference `distillers/NST.py:8-62`).

Polynomial-kernel (k(a,b) = (a.b)^2) MMD between channel-normalised spatial
maps, per stage.  The three kernel means are batched Gram products
(``bmm`` on MFMA through hipBLASLt): mean_ij (f_i . g_j)^2 = ||F G^T||_F^2 / C^2.
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class NST(Distiller):
    teacher_needs = ("feats",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.NST.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.NST.LOSS.FEAT_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_feat = self.feat_loss_weight * FL.nst_loss(
            feature_student["feats"][1:], feature_teacher["feats"][1:])
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
