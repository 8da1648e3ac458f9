"""Self-supervised KD with SVD (reference `distillers/KDSVD.py:8-98`).

Batched SVD of every stage (rocSOLVER through torch.linalg), sign-aligned
right singular vectors, RBF between consecutive stages, L2.
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class KDSVD(Distiller):
    teacher_needs = ("feats",)
    graph_capturable = False  # rocSOLVER batched SVD synchronises with the host

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.k = cfg.KDSVD.K
        self.ce_loss_weight = cfg.KDSVD.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.KDSVD.LOSS.FEAT_WEIGHT

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        loss_feat = self.feat_loss_weight * FL.kdsvd_loss(
            feature_student["feats"][1:], feature_teacher["feats"][1:], self.k)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
