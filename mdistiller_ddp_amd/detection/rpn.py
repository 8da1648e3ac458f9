"""Region proposal network: Detectron2's ``RPN`` + ``StandardRPNHead`` +
``DefaultAnchorGenerator``, the proposal generator of every reference
detection config (`detection/configs/Base-Distillation.yaml:9-20`).

Proposal selection runs on the device: per-level top-k, box decoding, and
one batched NMS launch per image over all levels (``ops/csrc/det.hip``,
level index folded into the box offsets) capped at the post-NMS top-k.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from .backbone import Conv2d
from .boxes import Box2BoxTransform, Matcher, clip_boxes, nonempty, pairwise_iou, subsample_labels
from .ops import batched_nms
from .structures import Instances


def smooth_l1_sum(x, y, beta: float):
    d = (x.float() - y.float()).abs()
    if beta < 1e-5:
        return d.sum()
    return torch.where(d < beta, 0.5 * d * d / beta, d - 0.5 * beta).sum()


def _broadcast(params, n):
    params = [list(p) for p in params]
    if len(params) == 1:
        return params * n
    assert len(params) == n, f"anchor params for {len(params)} levels, {n} feature maps"
    return params


class DefaultAnchorGenerator(nn.Module):
    def __init__(self, sizes, aspect_ratios, strides, offset=0.0):
        super().__init__()
        n = len(strides)
        self.strides = [int(s) for s in strides]
        self.offset = float(offset)
        self.cell_anchors = [self._cell(s, a) for s, a in
                             zip(_broadcast(sizes, n), _broadcast(aspect_ratios, n))]
        self._cache = {}

    @staticmethod
    def _cell(sizes, ratios):
        out = []
        for size in sizes:
            area = float(size) ** 2
            for r in ratios:
                w = math.sqrt(area / r)
                h = r * w
                out.append([-w / 2.0, -h / 2.0, w / 2.0, h / 2.0])
        return torch.tensor(out, dtype=torch.float32)

    @property
    def num_anchors(self):
        return [len(c) for c in self.cell_anchors]

    def forward(self, features):
        out = []
        for f, stride, cell in zip(features, self.strides, self.cell_anchors):
            h, w = int(f.shape[-2]), int(f.shape[-1])
            key = (h, w, stride, str(f.device))
            a = self._cache.get(key)
            if a is None:
                sx = torch.arange(0, w, dtype=torch.float32, device=f.device) * stride + self.offset * stride
                sy = torch.arange(0, h, dtype=torch.float32, device=f.device) * stride + self.offset * stride
                yy, xx = torch.meshgrid(sy, sx, indexing="ij")
                xx, yy = xx.reshape(-1), yy.reshape(-1)
                shifts = torch.stack((xx, yy, xx, yy), dim=1)
                a = (shifts.view(-1, 1, 4) + cell.to(f.device).view(1, -1, 4)).reshape(-1, 4)
                self._cache[key] = a
            out.append(a)
        return out


class StandardRPNHead(nn.Module):
    def __init__(self, in_channels, num_anchors, box_dim=4):
        super().__init__()
        self.conv = Conv2d(in_channels, in_channels, 3, 1, 1, activation="relu")
        self.objectness_logits = nn.Conv2d(in_channels, num_anchors, 1)
        self.anchor_deltas = nn.Conv2d(in_channels, num_anchors * box_dim, 1)
        for layer in (self.conv, self.objectness_logits, self.anchor_deltas):
            nn.init.normal_(layer.weight, std=0.01)
            nn.init.constant_(layer.bias, 0)

    def forward(self, features):
        logits, deltas = [], []
        for x in features:
            t = self.conv(x)
            logits.append(self.objectness_logits(t))
            deltas.append(self.anchor_deltas(t))
        return logits, deltas


@torch.no_grad()
def find_top_rpn_proposals(proposals, logits, image_sizes, nms_thresh, pre_topk, post_topk,
                           min_size, training):
    N = len(image_sizes)
    dev = proposals[0].device
    bidx = torch.arange(N, device=dev)
    scores_l, props_l, lvl_l = [], [], []
    for lvl, (p, l) in enumerate(zip(proposals, logits)):
        k = min(int(pre_topk), l.shape[1])
        s, idx = l.float().topk(k, dim=1)
        scores_l.append(s)
        props_l.append(p[bidx[:, None], idx])
        lvl_l.append(torch.full((k,), lvl, dtype=torch.int64, device=dev))
    scores = torch.cat(scores_l, 1)
    props = torch.cat(props_l, 1)
    level_ids = torch.cat(lvl_l)
    results = []
    for n, size in enumerate(image_sizes):
        boxes, sc, lvl = props[n], scores[n], level_ids
        valid = torch.isfinite(boxes).all(dim=1) & torch.isfinite(sc)
        if not bool(valid.all()):
            if training:
                raise FloatingPointError("predicted boxes or scores contain Inf/NaN: training has diverged")
            boxes, sc, lvl = boxes[valid], sc[valid], lvl[valid]
        boxes = clip_boxes(boxes, size)
        keep = nonempty(boxes, min_size)
        if not bool(keep.all()):
            boxes, sc, lvl = boxes[keep], sc[keep], lvl[keep]
        keep = batched_nms(boxes, sc, lvl, nms_thresh, max_keep=int(post_topk))[:int(post_topk)]
        results.append(Instances(size, proposal_boxes=boxes[keep], objectness_logits=sc[keep]))
    return results


class RPN(nn.Module):
    def __init__(self, mcfg, input_shape):
        super().__init__()
        r = mcfg.RPN
        self.in_features = list(r.IN_FEATURES)
        shapes = [input_shape[f] for f in self.in_features]
        self.anchor_generator = DefaultAnchorGenerator(mcfg.ANCHOR_GENERATOR.SIZES,
                                                       mcfg.ANCHOR_GENERATOR.ASPECT_RATIOS,
                                                       [s.stride for s in shapes],
                                                       mcfg.ANCHOR_GENERATOR.OFFSET)
        na = self.anchor_generator.num_anchors
        assert len(set(na)) == 1, "every level needs the same number of anchors"
        assert len(set(s.channels for s in shapes)) == 1
        self.rpn_head = StandardRPNHead(shapes[0].channels, na[0])
        self.anchor_matcher = Matcher(r.IOU_THRESHOLDS, r.IOU_LABELS, allow_low_quality_matches=True)
        self.box2box_transform = Box2BoxTransform(r.BBOX_REG_WEIGHTS)
        self.batch_size_per_image = int(r.BATCH_SIZE_PER_IMAGE)
        self.positive_fraction = float(r.POSITIVE_FRACTION)
        self.pre_nms_topk = {True: r.PRE_NMS_TOPK_TRAIN, False: r.PRE_NMS_TOPK_TEST}
        self.post_nms_topk = {True: r.POST_NMS_TOPK_TRAIN, False: r.POST_NMS_TOPK_TEST}
        self.nms_thresh = float(r.NMS_THRESH)
        self.min_box_size = float(mcfg.PROPOSAL_GENERATOR.MIN_SIZE)
        self.smooth_l1_beta = float(r.SMOOTH_L1_BETA)
        self.loss_weight = {"loss_rpn_cls": float(r.LOSS_WEIGHT),
                            "loss_rpn_loc": float(r.BBOX_REG_LOSS_WEIGHT) * float(r.LOSS_WEIGHT)}

    def forward(self, images, features, gt_instances=None):
        feats = [features[f] for f in self.in_features]
        anchors = self.anchor_generator(feats)
        logits, deltas = self.rpn_head(feats)
        # (N, A, H, W) -> (N, H*W*A);  (N, A*4, H, W) -> (N, H*W*A, 4)
        logits = [s.permute(0, 2, 3, 1).reshape(s.shape[0], -1) for s in logits]
        deltas = [x.reshape(x.shape[0], -1, 4, x.shape[-2], x.shape[-1]).permute(0, 3, 4, 1, 2)
                  .reshape(x.shape[0], -1, 4) for x in deltas]
        losses = {}
        if self.training:
            assert gt_instances is not None, "RPN requires gt_instances in training"
            gt_labels, gt_boxes = self.label_and_sample_anchors(anchors, gt_instances)
            losses = self.losses(anchors, logits, gt_labels, deltas, gt_boxes)
        proposals = self.predict_proposals(anchors, logits, deltas, images.image_sizes)
        return proposals, losses

    @torch.no_grad()
    def label_and_sample_anchors(self, anchors, gt_instances):
        anchors = torch.cat(anchors, 0)
        gt_labels, matched = [], []
        for inst in gt_instances:
            gtb = inst.gt_boxes
            idx, lab = self.anchor_matcher(pairwise_iou(gtb, anchors))
            pos, neg = subsample_labels(lab, self.batch_size_per_image, self.positive_fraction, 0)
            lab = torch.full_like(lab, -1)
            lab[pos] = 1
            lab[neg] = 0
            gt_labels.append(lab)
            matched.append(gtb[idx].float() if len(gtb) else torch.zeros_like(anchors))
        return gt_labels, matched

    def losses(self, anchors, logits, gt_labels, deltas, gt_boxes):
        num_images = len(gt_labels)
        gt_labels = torch.stack(gt_labels)
        anchors = torch.cat(anchors, 0)
        gt_deltas = torch.stack([self.box2box_transform.get_deltas(anchors, k) for k in gt_boxes])
        pos = gt_labels == 1
        loc = smooth_l1_sum(torch.cat(deltas, dim=1)[pos], gt_deltas[pos], self.smooth_l1_beta)
        valid = gt_labels >= 0
        obj = F.binary_cross_entropy_with_logits(torch.cat(logits, dim=1)[valid].float(),
                                                 gt_labels[valid].float(), reduction="sum")
        norm = float(self.batch_size_per_image * num_images)
        return {"loss_rpn_cls": obj / norm * self.loss_weight["loss_rpn_cls"],
                "loss_rpn_loc": loc / norm * self.loss_weight["loss_rpn_loc"]}

    @torch.no_grad()
    def predict_proposals(self, anchors, logits, deltas, image_sizes):
        N = logits[0].shape[0]
        props = []
        for a, d in zip(anchors, deltas):
            d2 = d.reshape(-1, 4)
            a2 = a.unsqueeze(0).expand(N, -1, -1).reshape(-1, 4)
            props.append(self.box2box_transform.apply_deltas(d2, a2).view(N, -1, 4))
        return find_top_rpn_proposals(props, [l.detach() for l in logits], image_sizes, self.nms_thresh,
                                      self.pre_nms_topk[self.training], self.post_nms_topk[self.training],
                                      self.min_box_size, self.training)
