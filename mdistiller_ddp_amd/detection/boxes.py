"""Box geometry of the RCNN stack: IoU, the (dx, dy, dw, dh) box coder, the
IoU matcher and the balanced label sampler -- the Detectron2 semantics
(`detectron2.modeling.{box_regression, matcher, sampling}`) that the
reference's detectors are trained with (`detection/model/rcnn.py`)."""
from __future__ import annotations

import math

import torch

_DEFAULT_SCALE_CLAMP = math.log(1000.0 / 16)


def box_area(b: torch.Tensor) -> torch.Tensor:
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])


def pairwise_iou(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``[N, M]`` IoU of two box sets (0 where boxes do not overlap)."""
    a = a.float()
    b = b.float()
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = box_area(a)[:, None] + box_area(b)[None, :] - inter
    return torch.where(inter > 0, inter / union, torch.zeros((), dtype=inter.dtype, device=inter.device))


def clip_boxes(b: torch.Tensor, image_size) -> torch.Tensor:
    h, w = image_size
    x1 = b[:, 0].clamp(min=0, max=w)
    y1 = b[:, 1].clamp(min=0, max=h)
    x2 = b[:, 2].clamp(min=0, max=w)
    y2 = b[:, 3].clamp(min=0, max=h)
    return torch.stack((x1, y1, x2, y2), dim=-1)


def nonempty(b: torch.Tensor, threshold: float = 0.0) -> torch.Tensor:
    return ((b[:, 2] - b[:, 0]) > threshold) & ((b[:, 3] - b[:, 1]) > threshold)


class Box2BoxTransform:
    """R-CNN box coder: deltas are centre offsets / size and log size ratios,
    scaled by per-coordinate ``weights``."""

    def __init__(self, weights, scale_clamp: float = _DEFAULT_SCALE_CLAMP):
        self.weights = tuple(float(w) for w in weights)
        self.scale_clamp = scale_clamp

    def get_deltas(self, src: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        src = src.float()
        target = target.float()
        sw, sh = src[:, 2] - src[:, 0], src[:, 3] - src[:, 1]
        sx, sy = src[:, 0] + 0.5 * sw, src[:, 1] + 0.5 * sh
        tw, th = target[:, 2] - target[:, 0], target[:, 3] - target[:, 1]
        tx, ty = target[:, 0] + 0.5 * tw, target[:, 1] + 0.5 * th
        wx, wy, ww, wh = self.weights
        return torch.stack((wx * (tx - sx) / sw, wy * (ty - sy) / sh,
                            ww * torch.log(tw / sw), wh * torch.log(th / sh)), dim=1)

    def apply_deltas(self, deltas: torch.Tensor, boxes: torch.Tensor) -> torch.Tensor:
        deltas = deltas.float()
        boxes = boxes.to(deltas.dtype)
        w, h = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
        cx, cy = boxes[:, 0] + 0.5 * w, boxes[:, 1] + 0.5 * h
        wx, wy, ww, wh = self.weights
        dx = deltas[:, 0::4] / wx
        dy = deltas[:, 1::4] / wy
        dw = (deltas[:, 2::4] / ww).clamp(max=self.scale_clamp)
        dh = (deltas[:, 3::4] / wh).clamp(max=self.scale_clamp)
        pcx = dx * w[:, None] + cx[:, None]
        pcy = dy * h[:, None] + cy[:, None]
        pw = torch.exp(dw) * w[:, None]
        ph = torch.exp(dh) * h[:, None]
        out = torch.stack((pcx - 0.5 * pw, pcy - 0.5 * ph, pcx + 0.5 * pw, pcy + 0.5 * ph), dim=-1)
        return out.reshape(deltas.shape)


class Matcher:
    """Assign each prediction (column) the best ground truth (row) and a label
    from the IoU interval it falls into; optionally also promote, for every
    ground truth, the predictions it overlaps best (low-quality matches)."""

    def __init__(self, thresholds, labels, allow_low_quality_matches: bool = False):
        thresholds = [float(t) for t in thresholds]
        self.thresholds = [-float("inf")] + thresholds + [float("inf")]
        self.labels = [int(l) for l in labels]
        assert len(self.labels) == len(self.thresholds) - 1
        self.allow_low_quality_matches = allow_low_quality_matches

    def __call__(self, quality: torch.Tensor):
        if quality.numel() == 0:
            n = quality.shape[1]
            return (torch.zeros(n, dtype=torch.int64, device=quality.device),
                    torch.full((n,), self.labels[0], dtype=torch.int8, device=quality.device))
        vals, matches = quality.max(dim=0)
        labels = torch.ones(matches.shape, dtype=torch.int8, device=quality.device)
        for l, lo, hi in zip(self.labels, self.thresholds[:-1], self.thresholds[1:]):
            labels[(vals >= lo) & (vals < hi)] = l
        if self.allow_low_quality_matches:
            best, _ = quality.max(dim=1)
            _, pred = torch.nonzero(quality == best[:, None], as_tuple=True)
            labels[pred] = 1
        return matches, labels


def subsample_labels(labels: torch.Tensor, num_samples: int, positive_fraction: float, bg_label: int):
    """Random positive / negative index subsets (positives capped at the fraction)."""
    pos = torch.nonzero((labels != -1) & (labels != bg_label), as_tuple=True)[0]
    neg = torch.nonzero(labels == bg_label, as_tuple=True)[0]
    num_pos = min(pos.numel(), int(num_samples * positive_fraction))
    num_neg = min(neg.numel(), num_samples - num_pos)
    p1 = torch.randperm(pos.numel(), device=pos.device)[:num_pos]
    p2 = torch.randperm(neg.numel(), device=neg.device)[:num_neg]
    return pos[p1], neg[p2]
