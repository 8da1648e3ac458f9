"""Relational KD, CVPR 2019 (reference `distillers/RKD.py:8-84`).

Distance term: pairwise distances normalised by their mean, smooth-L1.
Angle term: cosines of all (i; j, k) angles via a batched Gram of the
normalised difference vectors, smooth-L1.
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class RKD(Distiller):
    teacher_needs = ("pooled",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.distance_weight = cfg.RKD.DISTANCE_WEIGHT
        self.angle_weight = cfg.RKD.ANGLE_WEIGHT
        self.ce_loss_weight = cfg.RKD.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.RKD.LOSS.FEAT_WEIGHT
        self.eps = cfg.RKD.PDIST.EPSILON
        self.squared = cfg.RKD.PDIST.SQUARED

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_rkd = self.feat_loss_weight * FL.rkd_loss(
            feature_student["pooled_feat"], feature_teacher["pooled_feat"], self.squared,
            self.eps, self.distance_weight, self.angle_weight)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_rkd}
