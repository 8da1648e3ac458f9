"""FitNets: hints for thin deep nets (reference `distillers/FitNet.py:9-48`).

A :class:`ConvReg` maps the student's hint-layer feature onto the teacher's
(the conv + BN + ReLU runs on the fused training conv kernels); loss = MSE.
On the GPU the MSE value and its gradient come from one fused pass
(csrc/feat.hip ``mda_ofd_loss`` with no margin: bf16 NHWC in, fixed-order
partial sums).  The regressor is a distiller-owned module, so it is trained
and its gradients are all-reduced with the student's (flat buffer).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._base import Distiller
from ._common import ConvReg, get_feat_shapes
from ..ops import losses as L


class _HintMSEHIP(torch.autograd.Function):
    """weight * mean((s - t)^2) and its d/ds in one launch."""

    @staticmethod
    def forward(ctx, source, target, weight):
        from ..ops import _ext
        from ..ops.losses import workspace
        N, C, H, W = source.shape
        s = source.contiguous(memory_format=torch.channels_last)
        t = target.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        grad = torch.empty_like(s)
        loss = torch.empty(1, dtype=torch.float32, device=s.device)
        ws = workspace(s.device)
        _ext.call("mda_ofd_loss", s, t, None, grad, loss, ws.partial, ws.counter, N * H * W, C,
                  float(weight) / s.numel())
        ctx.save_for_backward(grad)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, go):
        (grad,) = ctx.saved_tensors
        return grad * go.to(grad.dtype), None, None


def hint_loss(f_s, f_t, weight):
    """`weight * F.mse_loss(f_s, f_t)` (reference `distillers/FitNet.py:41-43`)."""
    from ..ops.backend import hip_enabled_for
    if (hip_enabled_for(f_s) and f_s.dtype == torch.bfloat16 and f_s.dim() == 4
            and f_s.shape == f_t.shape and f_s.shape[1] % 8 == 0
            and f_s.is_contiguous(memory_format=torch.channels_last)):
        return _HintMSEHIP.apply(f_s, f_t, weight)
    return weight * F.mse_loss(f_s.float(), f_t.float())


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
        loss_feat = hint_loss(f_s, f_t, self.feat_loss_weight)
        return logits_student, {"loss_ce": loss_ce, "loss_kd": loss_feat}
