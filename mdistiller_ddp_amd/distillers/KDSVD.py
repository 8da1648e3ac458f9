"""Self-supervised KD with SVD (reference `distillers/KDSVD.py:8-98`).

Per-sample SVD of every stage, sign-aligned right singular vectors, RBF
between consecutive stages, L2.  The SVDs run as W x W Gram
eigendecompositions on a native Jacobi kernel (``ops/csrc/eig.hip``), so the
step captures into a hipGraph; shapes it does not cover fall back to
rocSOLVER's SVD (host-synchronising, eager).
"""
from __future__ import annotations

from ._base import Distiller
from ..ops import losses as L
from ..ops import feat_losses as FL


class KDSVD(Distiller):
    teacher_needs = ("feats",)
    # decided on the first step's feature shapes (see ``observe``)
    _capturable = True

    @property
    def graph_capturable(self) -> bool:
        return self._capturable

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
        g_s, g_t = feature_student["feats"][1:], feature_teacher["feats"][1:]
        if not FL.kdsvd_native_ok(g_s, g_t):
            self._capturable = False  # rocSOLVER path: eager steps
        loss_feat = self.feat_loss_weight * FL.kdsvd_loss(g_s, g_t, self.k)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
