"""Variational Information Distillation, CVPR 2019 (reference `distillers/VID.py:33-99`).

Per stage a 3 x (1x1 conv) regressor predicts the teacher feature's mean;
the loss is the Gaussian NLL with a learned per-channel softplus variance.

The per-channel ``log_scales`` are registered parameters here
(``nn.ParameterList``) so they are trained, checkpointed and moved with the
module; the reference keeps them in a plain Python list, so they never train
and never reach the GPU.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ._base import Distiller
from ._common import get_feat_shapes
from ..ops import losses as L
from ..ops import feat_losses as FL


def conv1x1(in_channels, out_channels, stride=1):
    return nn.Conv2d(in_channels, out_channels, kernel_size=1, padding=0, bias=False, stride=stride)


class VID(Distiller):
    teacher_needs = ("feats",)

    def __init__(self, student, teacher, cfg):
        super().__init__(student, teacher)
        self.ce_loss_weight = cfg.VID.LOSS.CE_WEIGHT
        self.feat_loss_weight = cfg.VID.LOSS.FEAT_WEIGHT
        self.init_pred_var = cfg.VID.INIT_PRED_VAR
        self.eps = cfg.VID.EPS
        s_shapes, t_shapes = get_feat_shapes(self.student, self.teacher, cfg.VID.INPUT_SIZE)
        self.init_vid_modules([s[1] for s in s_shapes[1:]], [s[1] for s in t_shapes[1:]])

    def init_vid_modules(self, s_channels, t_channels):
        self.regressors = nn.ModuleList()
        self.log_scales = nn.ParameterList()
        init = math.log(math.exp(self.init_pred_var - self.eps) - 1.0)
        for s, t in zip(s_channels, t_channels):
            self.regressors.append(nn.Sequential(conv1x1(s, t), nn.ReLU(), conv1x1(t, t), nn.ReLU(),
                                                 conv1x1(t, t)))
            self.log_scales.append(nn.Parameter(init * torch.ones(t)))

    def get_extra_parameters(self) -> int:
        return sum(p.numel() for p in self.regressors.parameters())

    def forward_train(self, image, target, **kwargs):
        t_out = self.teacher_forward(image)
        logits_student, feature_student = self.student(image)
        _, feature_teacher = t_out.get()
        loss_ce = L.ce(logits_student, target, self.ce_loss_weight)
        fs, ft = feature_student["feats"][1:], feature_teacher["feats"][1:]
        loss_vid = 0.0
        for i in range(len(fs)):
            loss_vid = loss_vid + FL.vid_loss(self.regressors[i], self.log_scales[i], fs[i], ft[i],
                                              self.eps)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": self.feat_loss_weight * loss_vid}
