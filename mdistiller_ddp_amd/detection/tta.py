"""Test-time augmentation for the detector (reference ``train_net.py:106-117``:
``GeneralizedRCNNWithTTA`` when ``TEST.AUG.ENABLED``).

Every image runs at each ``TEST.AUG.MIN_SIZES`` shortest edge (longest edge
capped at ``TEST.AUG.MAX_SIZE``), and horizontally flipped when
``TEST.AUG.FLIP``; boxes come back in original-image coordinates (the model's
own post-processing rescales to ``height`` / ``width``; flips are undone
here), are merged by class-wise NMS at ``MODEL.ROI_HEADS.NMS_THRESH_TEST`` and
cut to ``TEST.DETECTIONS_PER_IMAGE``.  Boxes only: the reference also
averages the mask logits of every augmentation for mask models; here a mask
model's TTA output carries no masks (box AP under TTA, mask AP without).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .data import resize_shape
from .ops import batched_nms
from .structures import Instances


class GeneralizedRCNNWithTTA(nn.Module):
    def __init__(self, cfg, model):
        super().__init__()
        self.model = model
        aug = cfg.TEST.AUG
        self.min_sizes = tuple(int(s) for s in aug.MIN_SIZES)
        self.max_size = int(aug.MAX_SIZE)
        self.flip = bool(aug.FLIP)
        self.nms_thresh = float(cfg.MODEL.ROI_HEADS.NMS_THRESH_TEST)
        self.max_dets = int(cfg.TEST.DETECTIONS_PER_IMAGE)

    def _augmented_inputs(self, x):
        img = x["image"]
        H0, W0 = int(x.get("height", img.shape[-2])), int(x.get("width", img.shape[-1]))
        for s in self.min_sizes:
            h, w, _ = resize_shape(img.shape[-2], img.shape[-1], s, self.max_size)
            im = F.interpolate(img[None].float(), size=(h, w), mode="bilinear",
                               align_corners=False)[0].round().clamp(0, 255).to(img.dtype)
            yield {"image": im, "height": H0, "width": W0}, False
            if self.flip:
                yield {"image": im.flip(-1), "height": H0, "width": W0}, True

    @torch.no_grad()
    def forward(self, batched_inputs):
        outs = []
        for x in batched_inputs:
            W0 = int(x.get("width", x["image"].shape[-1]))
            boxes, scores, classes = [], [], []
            for xi, flipped in self._augmented_inputs(x):
                r = self.model([xi])[0]["instances"]
                b = r.pred_boxes.float()
                if flipped:
                    b = torch.stack([W0 - b[:, 2], b[:, 1], W0 - b[:, 0], b[:, 3]], 1)
                boxes.append(b)
                scores.append(r.scores.float())
                classes.append(r.pred_classes)
            b = torch.cat(boxes)
            s = torch.cat(scores)
            c = torch.cat(classes)
            keep = batched_nms(b, s, c, self.nms_thresh)[: self.max_dets]
            H0 = int(x.get("height", x["image"].shape[-2]))
            inst = Instances((H0, W0), pred_boxes=b[keep], scores=s[keep], pred_classes=c[keep])
            outs.append({"instances": inst})
        return outs
