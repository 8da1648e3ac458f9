"""Second stage of the RCNN stack: Detectron2's ``StandardROIHeads`` with the
``FastRCNNConvFCHead`` box head, ``FastRCNNOutputLayers`` and the
``MaskRCNNConvUpsampleHead`` mask branch -- the ROI heads of every reference
detection config (`detection/configs/Base-Distillation.yaml:21-30`; the KD
meta-arch re-runs the box branch on the sampled proposals,
`detection/model/rcnn.py:152-157`).

Device-side design:

* :class:`ROIPooler` assigns every box its FPN level on the device and pools
  ALL levels in ONE multi-level ROIAlign launch (``ops/csrc/det.hip``,
  NHWC, level table in kernel arguments) instead of one launch per level
  plus a scatter.
* Mask targets are the gt bit masks crop-and-resized by the same kernel
  (C = 1), so no polygon rasterisation runs per step on the host.
* The box head's FCs are plain hipBLASLt GEMMs under bf16 autocast.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .backbone import Conv2d, c2_msra_fill, c2_xavier_fill, get_norm
from .boxes import Box2BoxTransform, Matcher, clip_boxes, nonempty, pairwise_iou, subsample_labels
from .ops import batched_nms, multilevel_roi_align, roi_align
from .rpn import smooth_l1_sum
from .structures import Instances


# ----------------------------------------------------------------------------- pooler
def assign_boxes_to_levels(boxes, min_level, max_level, canonical_box_size=224, canonical_level=4):
    """FPN level index (0-based from ``min_level``) of each box (FPN paper eq. 1)."""
    scale = ((boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])).clamp(min=0).sqrt()
    lvl = torch.floor(canonical_level + torch.log2(scale / canonical_box_size + 1e-8))
    return (lvl.clamp(min=min_level, max=max_level) - min_level).to(torch.int64)


def boxes_to_rois(box_lists):
    """[R, 5] (batch index, x1, y1, x2, y2) from per-image box tensors."""
    idx = [torch.full((len(b), 1), i, dtype=torch.float32, device=b.device) for i, b in enumerate(box_lists)]
    return torch.cat([torch.cat(idx, 0), torch.cat([b.float() for b in box_lists], 0)], 1)


class ROIPooler(nn.Module):
    def __init__(self, output_size, scales, sampling_ratio, pooler_type,
                 canonical_box_size=224, canonical_level=4):
        super().__init__()
        if isinstance(output_size, int):
            output_size = (output_size, output_size)
        assert pooler_type in ("ROIAlign", "ROIAlignV2"), f"pooler {pooler_type!r}"
        self.output_size = tuple(output_size)
        self.scales = [float(s) for s in scales]
        self.sampling_ratio = int(sampling_ratio)
        self.aligned = pooler_type == "ROIAlignV2"
        self.min_level = int(round(-math.log2(self.scales[0])))
        self.max_level = int(round(-math.log2(self.scales[-1])))
        self.canonical_box_size = canonical_box_size
        self.canonical_level = canonical_level

    def forward(self, features, box_lists):
        rois = boxes_to_rois(box_lists)
        if len(features) == 1:
            return roi_align(features[0], rois, self.output_size, self.scales[0], self.sampling_ratio,
                             self.aligned)
        levels = assign_boxes_to_levels(rois[:, 1:], self.min_level, self.max_level,
                                        self.canonical_box_size, self.canonical_level)
        return multilevel_roi_align(features, rois, levels, self.output_size, self.scales,
                                    self.sampling_ratio, self.aligned)


# ----------------------------------------------------------------------------- box branch
class FastRCNNConvFCHead(nn.Module):
    def __init__(self, in_channels, resolution, num_conv, conv_dim, num_fc, fc_dim, norm=""):
        super().__init__()
        self.conv_norm_relus = []
        c = in_channels
        for k in range(num_conv):
            conv = Conv2d(c, conv_dim, 3, padding=1, bias=not norm, norm=get_norm(norm, conv_dim),
                          activation="relu")
            c2_msra_fill(conv)
            self.add_module(f"conv{k + 1}", conv)
            self.conv_norm_relus.append(conv)
            c = conv_dim
        self.fcs = []
        d = c * resolution * resolution
        for k in range(num_fc):
            fc = nn.Linear(d, fc_dim)
            c2_xavier_fill(fc)
            self.add_module(f"fc{k + 1}", fc)
            self.fcs.append(fc)
            d = fc_dim
        self.output_size = d

    def forward(self, x):
        for conv in self.conv_norm_relus:
            x = conv(x)
        if self.fcs:
            x = x.flatten(1)
            for fc in self.fcs:
                x = F.relu(fc(x))
        return x


class FastRCNNOutputLayers(nn.Module):
    def __init__(self, input_size, num_classes, box2box_transform, cls_agnostic=False,
                 smooth_l1_beta=0.0, test_score_thresh=0.05, test_nms_thresh=0.5, test_topk=100,
                 loss_weight_box=1.0):
        super().__init__()
        self.num_classes = num_classes
        self.cls_score = nn.Linear(input_size, num_classes + 1)
        self.bbox_pred = nn.Linear(input_size, (1 if cls_agnostic else num_classes) * 4)
        nn.init.normal_(self.cls_score.weight, std=0.01)
        nn.init.normal_(self.bbox_pred.weight, std=0.001)
        for l in (self.cls_score, self.bbox_pred):
            nn.init.constant_(l.bias, 0)
        self.box2box_transform = box2box_transform
        self.smooth_l1_beta = smooth_l1_beta
        self.test_score_thresh = test_score_thresh
        self.test_nms_thresh = test_nms_thresh
        self.test_topk = test_topk
        self.loss_weight_box = loss_weight_box

    def forward(self, x):
        x = x.flatten(1)
        return self.cls_score(x), self.bbox_pred(x)

    def losses(self, predictions, proposals):
        scores, deltas = predictions
        gt_classes = torch.cat([p.gt_classes for p in proposals], 0)
        boxes = torch.cat([p.proposal_boxes for p in proposals], 0)
        gt_boxes = torch.cat([p.gt_boxes for p in proposals], 0)
        loss_cls = F.cross_entropy(scores.float(), gt_classes, reduction="mean")
        fg = torch.nonzero((gt_classes >= 0) & (gt_classes < self.num_classes), as_tuple=True)[0]
        gt_deltas = self.box2box_transform.get_deltas(boxes[fg], gt_boxes[fg])
        if deltas.shape[1] == 4:
            pred = deltas[fg]
        else:
            pred = deltas.view(deltas.shape[0], -1, 4)[fg, gt_classes[fg]]
        loss_box = smooth_l1_sum(pred, gt_deltas, self.smooth_l1_beta) / max(gt_classes.numel(), 1)
        return {"loss_cls": loss_cls, "loss_box_reg": loss_box * self.loss_weight_box}

    @torch.no_grad()
    def inference(self, predictions, proposals):
        scores, deltas = predictions
        n_per = [len(p) for p in proposals]
        boxes = torch.cat([p.proposal_boxes for p in proposals], 0)
        pred = self.box2box_transform.apply_deltas(deltas.float(), boxes)
        probs = F.softmax(scores.float(), dim=-1)
        out = []
        for b, s, p in zip(pred.split(n_per), probs.split(n_per), proposals):
            out.append(fast_rcnn_inference_single_image(b, s, p.image_size, self.test_score_thresh,
                                                        self.test_nms_thresh, self.test_topk))
        return out


def fast_rcnn_inference_single_image(boxes, scores, image_size, score_thresh, nms_thresh, topk):
    valid = torch.isfinite(boxes).all(dim=1) & torch.isfinite(scores).all(dim=1)
    if not bool(valid.all()):
        boxes, scores = boxes[valid], scores[valid]
    scores = scores[:, :-1]
    K = scores.shape[1]
    boxes = clip_boxes(boxes.reshape(-1, 4), image_size).view(-1, boxes.shape[1] // 4, 4)
    if boxes.shape[1] == 1:
        boxes = boxes.expand(-1, K, -1)
    keep_mask = scores > score_thresh
    idx = keep_mask.nonzero()
    b = boxes[idx[:, 0], idx[:, 1]]
    s = scores[keep_mask]
    keep = batched_nms(b, s, idx[:, 1], nms_thresh)
    if topk >= 0:
        keep = keep[:topk]
    return Instances(image_size, pred_boxes=b[keep], scores=s[keep], pred_classes=idx[keep, 1])


# ----------------------------------------------------------------------------- mask branch
class MaskRCNNConvUpsampleHead(nn.Module):
    def __init__(self, in_channels, num_classes, conv_dim, num_conv, norm="", cls_agnostic=False):
        super().__init__()
        self.conv_norm_relus = []
        c = in_channels
        for k in range(num_conv):
            conv = Conv2d(c, conv_dim, 3, 1, 1, bias=not norm, norm=get_norm(norm, conv_dim),
                          activation="relu")
            c2_msra_fill(conv)
            self.add_module(f"mask_fcn{k + 1}", conv)
            self.conv_norm_relus.append(conv)
            c = conv_dim
        self.deconv = nn.ConvTranspose2d(c, conv_dim, 2, 2)
        c2_msra_fill(self.deconv)
        self.predictor = nn.Conv2d(conv_dim, 1 if cls_agnostic else num_classes, 1)
        nn.init.normal_(self.predictor.weight, std=0.001)
        nn.init.constant_(self.predictor.bias, 0)

    def forward(self, x):
        for conv in self.conv_norm_relus:
            x = conv(x)
        return self.predictor(F.relu(self.deconv(x)))


def mask_rcnn_loss(pred_mask_logits, instances):
    """Per-pixel BCE of the gt-class mask logit against the gt mask
    crop-and-resized onto each foreground proposal (Detectron2 semantics)."""
    M = pred_mask_logits.shape[-1]
    cls_agnostic = pred_mask_logits.shape[1] == 1
    targets, classes = [], []
    for inst in instances:
        if len(inst) == 0:
            continue
        if not cls_agnostic:
            classes.append(inst.gt_classes)
        # gt_masks: [G, H, W] bit masks; gt_mask_index picks the matched gt of each proposal
        masks = inst.gt_masks[inst.gt_mask_index].unsqueeze(1).float()
        rois = torch.cat([torch.arange(len(inst), device=masks.device, dtype=torch.float32)[:, None],
                          inst.proposal_boxes.float()], 1)
        targets.append(roi_align(masks, rois, (M, M), 1.0, 0, True).squeeze(1))
    if not targets:
        return pred_mask_logits.sum() * 0
    gt = (torch.cat(targets, 0) >= 0.5).float()
    if cls_agnostic:
        logits = pred_mask_logits[:, 0]
    else:
        cls = torch.cat(classes, 0)
        logits = pred_mask_logits[torch.arange(len(cls), device=cls.device), cls]
    return F.binary_cross_entropy_with_logits(logits.float(), gt, reduction="mean")


def mask_rcnn_inference(pred_mask_logits, pred_instances):
    cls_agnostic = pred_mask_logits.shape[1] == 1
    if cls_agnostic:
        probs = pred_mask_logits.float().sigmoid()
    else:
        cls = torch.cat([i.pred_classes for i in pred_instances])
        probs = pred_mask_logits[torch.arange(len(cls), device=cls.device), cls][:, None].float().sigmoid()
    for p, inst in zip(probs.split([len(i) for i in pred_instances]), pred_instances):
        inst.pred_masks = p


# ----------------------------------------------------------------------------- ROI heads
class StandardROIHeads(nn.Module):
    def __init__(self, mcfg, input_shape):
        super().__init__()
        rh, bh, mh = mcfg.ROI_HEADS, mcfg.ROI_BOX_HEAD, mcfg.ROI_MASK_HEAD
        self.num_classes = int(rh.NUM_CLASSES)
        self.batch_size_per_image = int(rh.BATCH_SIZE_PER_IMAGE)
        self.positive_fraction = float(rh.POSITIVE_FRACTION)
        self.proposal_append_gt = bool(rh.PROPOSAL_APPEND_GT)
        self.proposal_matcher = Matcher(rh.IOU_THRESHOLDS, rh.IOU_LABELS, allow_low_quality_matches=False)
        self.in_features = self.box_in_features = list(rh.IN_FEATURES)
        scales = [1.0 / input_shape[f].stride for f in self.in_features]
        C = input_shape[self.in_features[0]].channels
        self.box_pooler = ROIPooler(bh.POOLER_RESOLUTION, scales, bh.POOLER_SAMPLING_RATIO, bh.POOLER_TYPE)
        self.box_head = FastRCNNConvFCHead(C, int(bh.POOLER_RESOLUTION), int(bh.NUM_CONV), int(bh.CONV_DIM),
                                           int(bh.NUM_FC), int(bh.FC_DIM), bh.NORM)
        self.box_predictor = FastRCNNOutputLayers(
            self.box_head.output_size, self.num_classes, Box2BoxTransform(bh.BBOX_REG_WEIGHTS),
            bool(bh.CLS_AGNOSTIC_BBOX_REG), float(bh.SMOOTH_L1_BETA), float(rh.SCORE_THRESH_TEST),
            float(rh.NMS_THRESH_TEST), 100, float(bh.BBOX_REG_LOSS_WEIGHT))
        self.mask_on = bool(mcfg.MASK_ON)
        if self.mask_on:
            self.mask_in_features = self.in_features
            self.mask_pooler = ROIPooler(mh.POOLER_RESOLUTION, scales, mh.POOLER_SAMPLING_RATIO,
                                         mh.POOLER_TYPE)
            self.mask_head = MaskRCNNConvUpsampleHead(C, self.num_classes, int(mh.CONV_DIM),
                                                      int(mh.NUM_CONV), mh.NORM, bool(mh.CLS_AGNOSTIC_MASK))

    def set_test_topk(self, k: int) -> None:
        self.box_predictor.test_topk = int(k)

    @torch.no_grad()
    def label_and_sample_proposals(self, proposals, targets):
        out = []
        for props, tgt in zip(proposals, targets):
            boxes = props.proposal_boxes
            if self.proposal_append_gt:
                boxes = torch.cat([boxes, tgt.gt_boxes.to(boxes.dtype)], 0)
            has_gt = len(tgt) > 0
            iou = pairwise_iou(tgt.gt_boxes, boxes)
            idx, lab = self.proposal_matcher(iou)
            if has_gt:
                cls = tgt.gt_classes[idx].clone()
                cls[lab == 0] = self.num_classes
                cls[lab == -1] = -1
            else:
                cls = torch.full_like(idx, self.num_classes)
            pos, neg = subsample_labels(cls, self.batch_size_per_image, self.positive_fraction,
                                        self.num_classes)
            sel = torch.cat([pos, neg])
            fields = dict(proposal_boxes=boxes[sel], gt_classes=cls[sel])
            fields["gt_boxes"] = (tgt.gt_boxes[idx[sel]].float() if has_gt
                                  else torch.zeros((len(sel), 4), device=boxes.device))
            if tgt.has("gt_masks"):
                fields["gt_mask_index"] = idx[sel]
            inst = Instances(props.image_size, **fields)
            if tgt.has("gt_masks"):
                object.__setattr__(inst, "gt_masks", tgt.gt_masks)  # per-image, not per-box
            out.append(inst)
        return out

    def _box_predictions(self, features, proposals):
        feats = [features[f] for f in self.box_in_features]
        x = self.box_pooler(feats, [p.proposal_boxes for p in proposals])
        return self.box_predictor(self.box_head(x))

    def forward(self, images, features, proposals, targets=None):
        if self.training:
            assert targets is not None
            proposals = self.label_and_sample_proposals(proposals, targets)
            preds = self._box_predictions(features, proposals)
            losses = self.box_predictor.losses(preds, proposals)
            if self.mask_on:
                losses.update(self._forward_mask(features, proposals))
            return proposals, losses
        preds = self._box_predictions(features, proposals)
        results = self.box_predictor.inference(preds, proposals)
        return self.forward_with_given_boxes(features, results), {}

    def forward_with_given_boxes(self, features, instances):
        if self.mask_on:
            feats = [features[f] for f in self.mask_in_features]
            x = self.mask_pooler(feats, [i.pred_boxes for i in instances])
            mask_rcnn_inference(self.mask_head(x), instances)
        return instances

    def _forward_mask(self, features, proposals):
        fg = []
        for p in proposals:
            k = torch.nonzero((p.gt_classes >= 0) & (p.gt_classes < self.num_classes), as_tuple=True)[0]
            inst = p[k]
            object.__setattr__(inst, "gt_masks", p.__dict__["gt_masks"])
            fg.append(inst)
        feats = [features[f] for f in self.mask_in_features]
        x = self.mask_pooler(feats, [p.proposal_boxes for p in fg])
        return {"loss_mask": mask_rcnn_loss(self.mask_head(x), fg)}


def build_roi_heads(mcfg, input_shape):
    name = mcfg.ROI_HEADS.NAME
    if name != "StandardROIHeads":
        raise NotImplementedError(f"ROI heads {name!r} (every reference config uses StandardROIHeads)")
    return StandardROIHeads(mcfg, input_shape)
