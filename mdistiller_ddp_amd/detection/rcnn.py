"""Meta-architectures: ``GeneralizedRCNN`` (the teacher, and a plain student)
and ``RCNNKD`` -- the student Faster/Mask R-CNN distilled from a frozen
teacher (reference `detection/model/rcnn.py:35-306`,
`detection/model/teacher/teacher.py:8-27`, `detection/model/reviewkd.py`).

KD types (``cfg.KD.TYPE``):

* ``DKD``: the teacher's ROI box branch is run on the STUDENT's sampled
  proposals and the two (K+1)-way logits go through the fused DKD loss
  kernel with the sampled gt classes as targets (`rcnn.py:26-33,196-203`).
* ``ReviewKD``: the student's FPN maps pass the 5-stage ABF review chain and
  are matched to the teacher's FPN maps with the HCL pyramid loss
  (`rcnn.py:204-210`, `reviewkd.py:5-92`).
* ``ReviewDKD``: both.

MI355X specifics: the frozen teacher backbone runs under ``no_grad`` with its
BNs folded into packed MFMA conv weights; when ``RUNTIME.TEACHER_STREAM`` is
set it is launched on a side HIP stream so it overlaps the student's
backbone + RPN (joined before the first kernel that reads teacher output).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import losses as L
from ..ops.nn import conv_bn_act
from .backbone import build_backbone, damp_residual_branches
from .roi_heads import build_roi_heads
from .rpn import RPN
from .structures import ImageList, Instances


# ----------------------------------------------------------------------------- ReviewKD (detection)
class ABF(nn.Module):
    """Attention-based fusion of one FPN level with the (upsampled) residual
    of the deeper level (`reviewkd.py:5-39`)."""

    def __init__(self, in_channel, mid_channel, out_channel, fuse):
        super().__init__()
        self.conv1 = nn.Sequential(nn.Conv2d(in_channel, mid_channel, 1, bias=False),
                                   nn.BatchNorm2d(mid_channel))
        self.conv2 = nn.Sequential(nn.Conv2d(mid_channel, out_channel, 3, 1, 1, bias=False),
                                   nn.BatchNorm2d(out_channel))
        self.att_conv = (nn.Sequential(nn.Conv2d(mid_channel * 2, 2, 1), nn.Sigmoid()) if fuse else None)
        nn.init.kaiming_uniform_(self.conv1[0].weight, a=1)
        nn.init.kaiming_uniform_(self.conv2[0].weight, a=1)

    def forward(self, x, y=None):
        n, _, h, w = x.shape
        x = conv_bn_act(x, self.conv1[0], self.conv1[1], "none")[0]
        if self.att_conv is not None:
            y = F.interpolate(y, (h, w), mode="nearest")
            z = torch.sigmoid(self.att_conv[0](torch.cat([x, y], 1)))
            x = x * z[:, 0:1] + y * z[:, 1:2]
        return conv_bn_act(x, self.conv2[0], self.conv2[1], "none")[0], x


class ReviewKDTrans(nn.Module):
    def __init__(self, in_channels, out_channels, mid_channel):
        super().__init__()
        abfs = [ABF(c, mid_channel, o, i < len(in_channels) - 1)
                for i, (c, o) in enumerate(zip(in_channels, out_channels))]
        self.abfs = nn.ModuleList(abfs[::-1])

    def forward(self, feats):
        x = feats[::-1]
        out, res = self.abfs[0](x[0])
        results = [out]
        for f, abf in zip(x[1:], self.abfs[1:]):
            out, res = abf(f, res)
            results.insert(0, out)
        return results


def build_kd_trans(kd_cfg=None, channels=256, levels=5):
    """5 x ABF(256 -> 256, mid 256) over p2..p6 (`reviewkd.py:68-73`)."""
    return ReviewKDTrans([channels] * levels, [channels] * levels, channels)


def hcl(fstudent, fteacher):
    """Hierarchical context loss, detection variant: pyramid levels 4/2/1
    skipped when not smaller than the map (`reviewkd.py:75-92`)."""
    total = 0.0
    for fs, ft in zip(fstudent, fteacher):
        h = fs.shape[2]
        fs, ft = fs.float(), ft.float()
        loss = F.mse_loss(fs, ft)
        cnt, tot = 1.0, 1.0
        for l in (4, 2, 1):
            if l >= h:
                continue
            cnt /= 2.0
            loss = loss + F.mse_loss(F.adaptive_avg_pool2d(fs, (l, l)), F.adaptive_avg_pool2d(ft, (l, l))) * cnt
            tot += cnt
        total = total + loss / tot
    return total


def rcnn_dkd_loss(stu_predictions, tea_predictions, gt_classes, alpha, beta, temperature):
    """DKD on the ROI classification logits (`rcnn.py:26-33`)."""
    target = torch.cat(tuple(gt_classes), 0).reshape(-1)
    return {"loss_dkd": L.dkd_loss(stu_predictions[0].float(), tea_predictions[0].float(), target,
                                   alpha, beta, temperature)}


# ----------------------------------------------------------------------------- meta-archs
def detector_postprocess(results: Instances, out_h, out_w):
    """Rescale predictions from the network input size to (out_h, out_w)."""
    sy = out_h / results.image_size[0]
    sx = out_w / results.image_size[1]
    out = Instances((out_h, out_w), **results.get_fields())
    if out.has("pred_boxes"):
        b = out.pred_boxes.clone()
        b[:, 0::2] *= sx
        b[:, 1::2] *= sy
        b = torch.stack([b[:, 0].clamp(0, out_w), b[:, 1].clamp(0, out_h),
                         b[:, 2].clamp(0, out_w), b[:, 3].clamp(0, out_h)], 1)
        keep = ((b[:, 2] - b[:, 0]) > 0) & ((b[:, 3] - b[:, 1]) > 0)
        out.set("pred_boxes", b)
        out = out[keep]
    if out.has("pred_masks") and len(out):
        m = out.pred_masks  # [R, 1, M, M] in-box masks -> full-image bit masks
        out.set("pred_masks", paste_masks_in_image(m[:, 0], out.pred_boxes, (out_h, out_w)))
    return out


def paste_masks_in_image(masks, boxes, image_shape, threshold=0.5):
    """Resample [R, M, M] in-box mask probabilities into [R, H, W] bit masks
    (grid_sample over the whole image; boxes in image pixels)."""
    H, W = image_shape
    R = masks.shape[0]
    if R == 0:
        return masks.new_zeros((0, H, W), dtype=torch.bool)
    ys = torch.arange(H, device=masks.device, dtype=torch.float32) + 0.5
    xs = torch.arange(W, device=masks.device, dtype=torch.float32) + 0.5
    x0, y0, x1, y1 = [boxes[:, i:i + 1].float() for i in range(4)]
    gx = (xs[None] - x0) / (x1 - x0) * 2 - 1
    gy = (ys[None] - y0) / (y1 - y0) * 2 - 1
    grid = torch.stack([gx[:, None, :].expand(R, H, W), gy[:, :, None].expand(R, H, W)], dim=3)
    out = F.grid_sample(masks[:, None].float(), grid, align_corners=False)
    return out[:, 0] >= threshold


class GeneralizedRCNN(nn.Module):
    """backbone + RPN + ROI heads from one model config node."""

    def __init__(self, mcfg, input_format="BGR"):
        super().__init__()
        self.backbone = build_backbone(mcfg)
        shapes = self.backbone.output_shape()
        self.proposal_generator = RPN(mcfg, shapes)
        self.roi_heads = build_roi_heads(mcfg, shapes)
        self.input_format = input_format
        self.register_buffer("pixel_mean", torch.tensor(mcfg.PIXEL_MEAN, dtype=torch.float32).view(-1, 1, 1), False)
        self.register_buffer("pixel_std", torch.tensor(mcfg.PIXEL_STD, dtype=torch.float32).view(-1, 1, 1), False)

    @property
    def device(self):
        return self.pixel_mean.device

    def preprocess_image(self, batched_inputs, mean=None, std=None, swap_rgb=False):
        mean = self.pixel_mean if mean is None else mean
        std = self.pixel_std if std is None else std
        imgs = []
        for x in batched_inputs:
            im = x["image"].to(self.device, non_blocking=True).float()
            im = (im - mean) / std
            if swap_rgb:
                im = im.flip(0)
            imgs.append(im)
        return ImageList.from_tensors(imgs, self.backbone.size_divisibility)

    def forward(self, batched_inputs):
        if not self.training:
            return self.inference(batched_inputs)
        images = self.preprocess_image(batched_inputs)
        gt = [x["instances"].to(self.device) for x in batched_inputs]
        features = self.backbone(images.tensor)
        proposals, losses = self.proposal_generator(images, features, gt)
        _, det_losses = self.roi_heads(images, features, proposals, gt)
        losses.update(det_losses)
        return losses

    @torch.no_grad()
    def inference(self, batched_inputs, do_postprocess=True):
        images = self.preprocess_image(batched_inputs)
        features = self.backbone(images.tensor)
        proposals, _ = self.proposal_generator(images, features, None)
        results, _ = self.roi_heads(images, features, proposals, None)
        if not do_postprocess:
            return results
        return [{"instances": detector_postprocess(r, x.get("height", s[0]), x.get("width", s[1]))}
                for r, x, s in zip(results, batched_inputs, images.image_sizes)]


def build_teacher(cfg) -> GeneralizedRCNN:
    """Frozen teacher from ``cfg.TEACHER`` (`teacher/teacher.py:15-27`)."""
    t = GeneralizedRCNN(cfg.TEACHER.MODEL, cfg.TEACHER.INPUT.FORMAT)
    for p in t.parameters():
        p.requires_grad_(False)
    t.eval()
    return t


class RCNNKD(GeneralizedRCNN):
    def __init__(self, cfg):
        super().__init__(cfg.MODEL, cfg.INPUT.FORMAT)
        self.kd_args = cfg.KD
        if self.kd_args.TYPE not in ("DKD", "ReviewKD", "ReviewDKD"):
            raise NotImplementedError(self.kd_args.TYPE)
        self.teacher = build_teacher(cfg)
        if self.kd_args.TYPE in ("ReviewKD", "ReviewDKD"):
            self.kd_trans = build_kd_trans(self.kd_args, cfg.MODEL.FPN.OUT_CHANNELS,
                                           len(self.backbone.output_shape()))
        self.teacher_input_format = cfg.TEACHER.INPUT.FORMAT
        self.register_buffer("teacher_pixel_mean",
                             torch.tensor(cfg.TEACHER.MODEL.PIXEL_MEAN, dtype=torch.float32).view(-1, 1, 1), False)
        self.register_buffer("teacher_pixel_std",
                             torch.tensor(cfg.TEACHER.MODEL.PIXEL_STD, dtype=torch.float32).view(-1, 1, 1), False)
        rt = getattr(cfg, "RUNTIME", None)
        if rt is not None and float(rt.RANDOM_INIT_DAMP) > 0 and not (
                cfg.MODEL.WEIGHTS and os.path.exists(cfg.MODEL.WEIGHTS)):
            damp_residual_branches(self, float(rt.RANDOM_INIT_DAMP))
        self.teacher_stream_on = bool(rt.TEACHER_STREAM) if rt is not None else False
        self._tstream = None

    def train(self, mode=True):
        super().train(mode)
        self.teacher.eval()  # frozen: BN statistics and proposals in eval mode
        return self

    def student_parameters(self):
        return [p for n, p in self.named_parameters() if not n.startswith("teacher.") and p.requires_grad]

    @staticmethod
    def forward_pure_roi_head(roi_head, features, proposals):
        return roi_head._box_predictions(features, proposals)

    def _teacher_features(self, batched_inputs):
        with torch.no_grad():
            timgs = self.preprocess_image(batched_inputs, self.teacher_pixel_mean, self.teacher_pixel_std,
                                          swap_rgb=self.input_format != self.teacher_input_format)
            return self.teacher.backbone(timgs.tensor)

    def forward(self, batched_inputs):
        if not self.training:
            return self.inference(batched_inputs)
        images = self.preprocess_image(batched_inputs)
        gt = [x["instances"].to(self.device) for x in batched_inputs]
        side = self.teacher_stream_on and images.tensor.is_cuda
        if side:
            if self._tstream is None:
                self._tstream = torch.cuda.Stream(device=images.tensor.device)
            self._tstream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._tstream):
                t_features = self._teacher_features(batched_inputs)
        else:
            t_features = self._teacher_features(batched_inputs)
        features = self.backbone(images.tensor)
        proposals, proposal_losses = self.proposal_generator(images, features, gt)
        sampled, detector_losses = self.roi_heads(images, features, proposals, gt)
        if side:
            torch.cuda.current_stream().wait_stream(self._tstream)
            for v in t_features.values():
                v.record_stream(torch.cuda.current_stream())
        losses = {}
        kd = self.kd_args.TYPE
        if kd in ("DKD", "ReviewDKD"):
            stu = self.forward_pure_roi_head(self.roi_heads, features, sampled)
            with torch.no_grad():
                tea = self.forward_pure_roi_head(self.teacher.roi_heads, t_features, sampled)
            d = self.kd_args.DKD
            detector_losses.update(rcnn_dkd_loss(stu, tea, [x.gt_classes for x in sampled],
                                                 d.ALPHA, d.BETA, d.T))
        if kd in ("ReviewKD", "ReviewDKD"):
            s_feats = self.kd_trans([features[f] for f in features])
            losses["loss_reviewkd"] = hcl(s_feats, [t_features[f] for f in t_features]) \
                * self.kd_args.REVIEWKD.LOSS_WEIGHT
        losses.update(detector_losses)
        losses.update(proposal_losses)
        return losses


META_ARCH_REGISTRY = {"GeneralizedRCNN": lambda cfg: GeneralizedRCNN(cfg.MODEL, cfg.INPUT.FORMAT),
                      "RCNNKD": RCNNKD}


def build_model(cfg):
    name = cfg.MODEL.META_ARCHITECTURE
    if name not in META_ARCH_REGISTRY:
        raise NotImplementedError(f"meta-architecture {name!r}")
    return META_ARCH_REGISTRY[name](cfg)
