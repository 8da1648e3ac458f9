"""FitNets: hints for thin deep nets (reference `distillers/FitNet.py:9-48`).

A :class:`ConvReg` maps the student's hint-layer feature onto the teacher's;
loss = MSE.  The regressor is a distiller-owned module, so it is trained and
its gradients are all-reduced with the student's (flat buffer).
"""
from __future__ import annotations

import torch.nn.functional as F

from ._base import Distiller
from ._common import ConvReg, get_feat_shapes
from ..ops import losses as L


class FitNet(Distiller):
    teacher_needs = ("feats",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.FITNET.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.FITNET.LOSS.FEAT_WEIGHT
        self.hint_layer = cfg.FITNET.HINT_LAYER
        s_shapes, t_shapes = get_feat_shapes(self.student, self.teacher, cfg.FITNET.INPUT_SIZE)
        self.conv_reg = ConvReg(s_shapes[self.hint_layer], t_shapes[self.hint_layer])

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        f_s = self.conv_reg(feature_student["feats"][self.hint_layer])
        f_t = feature_teacher["feats"][self.hint_layer]
        loss_feat = self.feat_loss_weight * F.mse_loss(f_s.float(), f_t.float())
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
