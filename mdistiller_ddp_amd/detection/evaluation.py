"""Dataset evaluators of the detection entry point.

The reference's ``Trainer.build_evaluator`` (``detection/train_net.py:55-104``)
picks Detectron2 evaluators by the dataset's ``evaluator_type``: COCO,
COCO-panoptic (sem-seg + COCO), LVIS, Pascal VOC, Cityscapes instance and
semantic segmentation, plain semantic segmentation, combined with
``DatasetEvaluators``.  Those live in Detectron2 (plus pycocotools / lvis-api
/ cityscapesscripts), none of which exists here, so this module implements
the metrics themselves, with the same evaluator protocol
(``reset`` / ``process(inputs, outputs)`` / ``evaluate``):

* box / mask AP with COCO matching (IoU 0.50:0.95, 101-point precision, area
  ranges), shared by COCO, LVIS (federated: negative and not-exhaustive
  category lists per image, 300 detections per image, APr / APc / APf) and
  Cityscapes instance masks;
* Pascal VOC AP (VOC2007 11-point or area metric, ``difficult`` boxes ignored)
  at IoU 0.50:0.95 -> AP, AP50, AP75 as Detectron2 reports them;
* semantic segmentation (confusion matrix -> mIoU, fwIoU, mACC, pACC and
  per-class IoU, ``ignore_label`` excluded); Cityscapes semantic = the same on
  the 19 train ids.

Inputs are per-image numpy dicts: predictions ``boxes`` [N, 4] xyxy,
``scores`` [N], ``classes`` [N] and optionally ``masks`` [N, H, W] bool;
ground truths ``boxes``, ``classes``, optionally ``masks``, ``difficult``,
``neg_category_ids`` and ``not_exhaustive_category_ids`` (LVIS).
"""
from __future__ import annotations

import numpy as np
import torch

COCO_IOUS = np.linspace(0.5, 0.95, 10)
AREA_RANGES = {"all": (0, 1e10), "small": (0, 32 ** 2), "medium": (32 ** 2, 96 ** 2), "large": (96 ** 2, 1e10)}


# ----------------------------------------------------------------------------- IoUs
def box_iou_np(a, b):
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    aa = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    ab = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    return inter / np.maximum(aa[:, None] + ab[None, :] - inter, 1e-12)


def _voc_iou(b, gb):
    """Pascal VOC IoU of one box against many, with the +1 pixel convention of
    Detectron2's ``voc_eval`` (inclusive integer pixel coordinates)."""
    ixmin = np.maximum(gb[:, 0], b[0])
    iymin = np.maximum(gb[:, 1], b[1])
    ixmax = np.minimum(gb[:, 2], b[2])
    iymax = np.minimum(gb[:, 3], b[3])
    iw = np.maximum(ixmax - ixmin + 1.0, 0.0)
    ih = np.maximum(iymax - iymin + 1.0, 0.0)
    inter = iw * ih
    uni = ((b[2] - b[0] + 1.0) * (b[3] - b[1] + 1.0)
           + (gb[:, 2] - gb[:, 0] + 1.0) * (gb[:, 3] - gb[:, 1] + 1.0) - inter)
    return inter / np.maximum(uni, 1e-12)


def mask_iou_np(a, b):
    """a [N, H, W], b [M, H, W] boolean masks -> [N, M] IoU."""
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    fa = a.reshape(len(a), -1).astype(np.float64)
    fb = b.reshape(len(b), -1).astype(np.float64)
    inter = fa @ fb.T
    union = fa.sum(1)[:, None] + fb.sum(1)[None, :] - inter
    return inter / np.maximum(union, 1e-12)


def _areas(d, iou_type):
    if iou_type == "segm":
        m = d["masks"]
        return m.reshape(len(m), -1).sum(1).astype(np.float64) if len(m) else np.zeros(0)
    b = d["boxes"]
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]) if len(b) else np.zeros(0)


# ----------------------------------------------------------------------------- COCO-style AP core
def _ap_101(tp, conf, n_gt):
    if n_gt == 0:
        return None
    if len(tp) == 0:
        return 0.0
    order = np.argsort(-conf, kind="mergesort")
    tp = tp[order]
    ctp, cfp = np.cumsum(tp), np.cumsum(1 - tp)
    rec = ctp / n_gt
    prec = ctp / np.maximum(ctp + cfp, np.spacing(1))
    prec = np.maximum.accumulate(prec[::-1])[::-1]
    idx = np.searchsorted(rec, np.linspace(0, 1, 101), side="left")
    q = np.where(idx < len(prec), prec[np.minimum(idx, len(prec) - 1)], 0.0)
    return float(q.mean())


def _greedy_match(iou, gign, thr, crowd=None):
    """COCO greedy matching of score-sorted detections to ground truths
    (non-ignored first); returns (matched gt index or -1) per detection.
    ``crowd``: iscrowd ground truths, which (as in pycocotools
    ``COCOeval.evaluateImg``) may absorb any number of detections."""
    D, G = iou.shape
    used = np.zeros(G, bool)
    order = np.argsort(gign, kind="mergesort")
    out = np.full(D, -1)
    for d in range(D):
        best, m = min(thr, 1 - 1e-10), -1
        for gi in order:
            if used[gi] and not (crowd is not None and crowd[gi]):
                continue
            if m > -1 and not gign[m] and gign[gi]:
                break
            if iou[d, gi] < best:
                continue
            best, m = iou[d, gi], gi
        if m >= 0:
            used[m] = True
            out[d] = m
    return out


def instance_ap(predictions, ground_truths, num_classes, *, iou_type="bbox", max_dets=100,
                per_image_max=False, ious=COCO_IOUS, area_ranges=AREA_RANGES, federated=False):
    """AP table ``[area][iou][class]`` (NaN where a class has no ground truth).

    ``per_image_max``: keep the ``max_dets`` best detections of an IMAGE over
    all classes (LVIS) instead of per class (COCO).  ``federated``: LVIS rules,
    a class is evaluated on an image only if it is annotated there or listed in
    ``neg_category_ids``; unmatched detections of a class in
    ``not_exhaustive_category_ids`` are ignored."""
    iou_fn = mask_iou_np if iou_type == "segm" else box_iou_np
    key = "masks" if iou_type == "segm" else "boxes"
    preds = []
    for p in predictions:
        o = np.argsort(-p["scores"], kind="mergesort")
        if per_image_max:
            o = o[:max_dets]
        preds.append({k: (v[o] if isinstance(v, np.ndarray) and len(v) == len(p["scores"]) else v)
                      for k, v in p.items()})
    out = {}
    for area_name, (lo, hi) in area_ranges.items():
        aps = np.full((len(ious), num_classes), np.nan)
        for c in range(num_classes):
            tps = [[] for _ in ious]
            n_gt = 0
            for p, g in zip(preds, ground_truths):
                gm = g["classes"] == c
                if federated:
                    neg = set(int(v) for v in g.get("neg_category_ids", ()))
                    if not gm.any() and c not in neg:
                        continue
                    not_exh = c in set(int(v) for v in g.get("not_exhaustive_category_ids", ()))
                else:
                    not_exh = False
                gobj = g[key][gm]
                # the annotation's ``area`` field when present (pycocotools), else
                # the box / mask area; inclusive upper bound like pycocotools
                ga = g["areas"][gm] if "areas" in g else _areas({key: gobj, "boxes": gobj}, iou_type)
                gign = (ga < lo) | (ga > hi)
                crowd = g["iscrowd"][gm].astype(bool) if "iscrowd" in g else None
                if crowd is not None:
                    gign = gign | crowd
                n_gt += int((~gign).sum())
                pm = p["classes"] == c
                pobj, ps = p[key][pm], p["scores"][pm]
                if not per_image_max:
                    pobj, ps = pobj[:max_dets], ps[:max_dets]
                if len(ps) == 0:
                    continue
                iou = iou_fn(pobj, gobj) if len(gobj) else np.zeros((len(ps), 0))
                pa = _areas({key: pobj, "boxes": pobj}, iou_type)
                if crowd is not None and crowd.any() and len(gobj):
                    # pycocotools: IoU with a crowd region = intersection / detection area
                    inter = iou * (pa[:, None] + _areas({key: gobj, "boxes": gobj}, iou_type)[None, :]) / (1 + iou)
                    iou = np.where(crowd[None, :], inter / np.maximum(pa[:, None], 1e-12), iou)
                for ti, t in enumerate(ious):
                    m = _greedy_match(iou, gign, t, crowd) if len(gobj) else np.full(len(ps), -1)
                    tp = (m >= 0).astype(np.float64)
                    ign = np.where(m >= 0, gign[np.maximum(m, 0)] if len(gobj) else False,
                                   (pa < lo) | (pa > hi) | not_exh)
                    keep = ~ign
                    tps[ti].append((tp[keep], ps[keep]))
            for ti in range(len(ious)):
                tp_all = np.concatenate([a for a, _ in tps[ti]]) if tps[ti] else np.zeros(0)
                cf_all = np.concatenate([b for _, b in tps[ti]]) if tps[ti] else np.zeros(0)
                ap = _ap_101(tp_all, cf_all, n_gt)
                if ap is not None:
                    aps[ti, c] = ap
        out[area_name] = aps
    return out


def _summarize(table, ious=COCO_IOUS, classes=None):
    def mean(a):
        a = a if classes is None else a[:, classes]
        return float(np.nanmean(a) * 100) if np.isfinite(a).any() else float("nan")
    res = {"AP": mean(table["all"])}
    i50 = int(np.argmin(np.abs(ious - 0.5)))
    i75 = int(np.argmin(np.abs(ious - 0.75)))
    res["AP50"] = mean(table["all"][i50:i50 + 1])
    res["AP75"] = mean(table["all"][i75:i75 + 1])
    for a in ("small", "medium", "large"):
        if a in table:
            res["AP" + a[0]] = mean(table[a])
    return res


def coco_instance_evaluate(predictions, ground_truths, num_classes, iou_type="bbox", max_dets=100):
    return _summarize(instance_ap(predictions, ground_truths, num_classes, iou_type=iou_type,
                                  max_dets=max_dets))


def lvis_evaluate(predictions, ground_truths, num_classes, iou_type="bbox", max_dets=300,
                  category_frequency=None):
    """LVIS AP (federated).  ``category_frequency``: class -> 'r' / 'c' / 'f'
    (the LVIS ``frequency`` field) adds APr / APc / APf."""
    table = instance_ap(predictions, ground_truths, num_classes, iou_type=iou_type, max_dets=max_dets,
                        per_image_max=True, federated=True)
    res = _summarize(table)
    if category_frequency:
        for f in ("r", "c", "f"):
            cl = [c for c, v in category_frequency.items() if v == f and c < num_classes]
            res["AP" + f] = _summarize(table, classes=cl)["AP"] if cl else float("nan")
    return res


# ----------------------------------------------------------------------------- Pascal VOC
def _voc_ap(rec, prec, use_07_metric):
    if use_07_metric:
        ap = 0.0
        for t in np.arange(0.0, 1.1, 0.1):
            p = np.max(prec[rec >= t]) if np.any(rec >= t) else 0.0
            ap += p / 11.0
        return float(ap)
    mrec = np.concatenate(([0.0], rec, [1.0]))
    mpre = np.concatenate(([0.0], prec, [0.0]))
    mpre = np.maximum.accumulate(mpre[::-1])[::-1]
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


def voc_class_ap(predictions, ground_truths, c, thr, use_07_metric=True):
    """VOC AP of class c: detections sorted by score over the whole set, each
    assigned to its max-IoU ground truth; ``difficult`` matches are ignored,
    repeated matches are false positives."""
    n_pos, dets = 0, []
    state = []
    for i, (p, g) in enumerate(zip(predictions, ground_truths)):
        gm = g["classes"] == c
        gb = g["boxes"][gm]
        diff = g["difficult"][gm].astype(bool) if "difficult" in g else np.zeros(len(gb), bool)
        n_pos += int((~diff).sum())
        state.append([gb, diff, np.zeros(len(gb), bool)])
        pm = p["classes"] == c
        for b, s in zip(p["boxes"][pm], p["scores"][pm]):
            dets.append((float(s), i, b))
    if n_pos == 0:
        return None
    dets.sort(key=lambda d: -d[0])
    tp = np.zeros(len(dets))
    fp = np.zeros(len(dets))
    for k, (_, i, b) in enumerate(dets):
        gb, diff, seen = state[i]
        if len(gb):
            iou = _voc_iou(b.astype(np.float64), gb.astype(np.float64))
            j = int(np.argmax(iou))
            if iou[j] > thr:
                if diff[j]:
                    continue
                if not seen[j]:
                    tp[k], seen[j] = 1, True
                else:
                    fp[k] = 1
                continue
        fp[k] = 1
    tp, fp = np.cumsum(tp), np.cumsum(fp)
    rec = tp / n_pos
    prec = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
    return _voc_ap(rec, prec, use_07_metric)


def voc_evaluate(predictions, ground_truths, num_classes, use_07_metric=True):
    """{"AP" (mean over IoU 0.50:0.95), "AP50", "AP75"} x 100, as Detectron2's
    ``PascalVOCDetectionEvaluator`` reports them."""
    per_t = {}
    for t in range(50, 100, 5):
        aps = [voc_class_ap(predictions, ground_truths, c, t / 100.0, use_07_metric) for c in range(num_classes)]
        aps = [a for a in aps if a is not None]
        per_t[t] = float(np.mean(aps) * 100) if aps else float("nan")
    return {"AP": float(np.mean(list(per_t.values()))), "AP50": per_t[50], "AP75": per_t[75]}


# ----------------------------------------------------------------------------- semantic segmentation
def semseg_confusion(pred, gt, num_classes, ignore_label=255):
    """pred / gt integer label maps of one image -> [K+1, K+1] counts (the
    last row/col collects ignored pixels, dropped by the metrics)."""
    pred = np.asarray(pred, dtype=np.int64).reshape(-1)
    gt = np.asarray(gt, dtype=np.int64).reshape(-1)
    gt = np.where(gt == ignore_label, num_classes, gt)
    pred = np.clip(pred, 0, num_classes)
    return np.bincount((num_classes + 1) * pred + gt, minlength=(num_classes + 1) ** 2).reshape(
        num_classes + 1, num_classes + 1)


def semseg_metrics(conf, class_names=None):
    """Detectron2 SemSegEvaluator metrics from a confusion matrix (pred x gt)."""
    K = conf.shape[0] - 1
    c = conf[:K, :K].astype(np.float64)
    tp = np.diag(c)
    pos_gt = c.sum(0)
    pos_pred = c.sum(1)
    acc_valid = pos_gt > 0
    iou_valid = (pos_gt + pos_pred) > 0
    with np.errstate(all="ignore"):
        acc = np.where(acc_valid, tp / np.maximum(pos_gt, 1), np.nan)
        iou = np.where(iou_valid, tp / np.maximum(pos_gt + pos_pred - tp, 1), np.nan)
    union = pos_gt + pos_pred - tp
    res = {
        "mIoU": float(np.nanmean(iou) * 100) if iou_valid.any() else float("nan"),
        "fwIoU": float(np.nansum(iou * (pos_gt / max(pos_gt.sum(), 1))) * 100),
        "mACC": float(np.nanmean(acc) * 100) if acc_valid.any() else float("nan"),
        "pACC": float(tp.sum() / max(pos_gt.sum(), 1) * 100),
    }
    for k in range(K):
        name = class_names[k] if class_names else str(k)
        res[f"IoU-{name}"] = float(iou[k] * 100) if union[k] > 0 else float("nan")
    return res


# ----------------------------------------------------------------------------- evaluator protocol
def _to_np(t):
    return t.detach().float().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def prediction_dict(inst):
    """Detector output ``Instances`` -> numpy prediction dict."""
    d = {"boxes": _to_np(inst.pred_boxes), "scores": _to_np(inst.scores),
         "classes": _to_np(inst.pred_classes).astype(np.int64)}
    if inst.has("pred_masks"):
        d["masks"] = _to_np(inst.pred_masks) > 0.5
    return d


def ground_truth_dict(x):
    """Dataset dict -> numpy ground truth at the ORIGINAL image size."""
    inst = x["instances"]
    sy = x.get("height", inst.image_size[0]) / inst.image_size[0]
    sx = x.get("width", inst.image_size[1]) / inst.image_size[1]
    d = {"boxes": _to_np(inst.gt_boxes) * np.array([sx, sy, sx, sy]),
         "classes": _to_np(inst.gt_classes).astype(np.int64)}
    if inst.has("gt_masks"):
        m = inst.gt_masks
        if m.shape[-2:] != (x.get("height", m.shape[-2]), x.get("width", m.shape[-1])):
            m = torch.nn.functional.interpolate(m[None].float(), size=(x["height"], x["width"]),
                                                mode="nearest")[0]
        d["masks"] = _to_np(m) > 0.5
    for k in ("difficult", "iscrowd", "neg_category_ids", "not_exhaustive_category_ids"):
        if k in x:
            d[k] = np.asarray(x[k])
    return d


class DatasetEvaluator:
    def reset(self):
        pass

    def process(self, inputs, outputs):
        raise NotImplementedError

    def evaluate(self):
        raise NotImplementedError

    def _gather(self, items):
        from ..parallel.dist import get_world_size
        if get_world_size() > 1:
            import torch.distributed as dist
            allv = [None] * get_world_size()
            dist.all_gather_object(allv, items)
            return [i for r in allv for i in r]
        return items


class _InstanceEvaluator(DatasetEvaluator):
    def __init__(self, num_classes, tasks=("bbox",)):
        self.num_classes = num_classes
        self.tasks = tuple(tasks)
        self.reset()

    def reset(self):
        self._preds, self._gts = [], []

    def process(self, inputs, outputs):
        for x, o in zip(inputs, outputs):
            self._preds.append(prediction_dict(o["instances"]))
            self._gts.append(ground_truth_dict(x))

    def _collect(self):
        return self._gather(self._preds), self._gather(self._gts)


class COCOEvaluator(_InstanceEvaluator):
    def __init__(self, num_classes, tasks=("bbox",), max_dets=100):
        self.max_dets = max_dets
        super().__init__(num_classes, tasks)

    def evaluate(self):
        preds, gts = self._collect()
        segm_ok = all("masks" in p for p in preds) and all("masks" in g for g in gts)
        return {t: coco_instance_evaluate(preds, gts, self.num_classes, t, self.max_dets)
                for t in self.tasks if t == "bbox" or segm_ok}


class LVISEvaluator(_InstanceEvaluator):
    def __init__(self, num_classes, tasks=("bbox",), max_dets=300, category_frequency=None):
        self.max_dets = max_dets
        self.category_frequency = category_frequency
        super().__init__(num_classes, tasks)

    def evaluate(self):
        preds, gts = self._collect()
        return {t: lvis_evaluate(preds, gts, self.num_classes, t, self.max_dets, self.category_frequency)
                for t in self.tasks}


class PascalVOCDetectionEvaluator(_InstanceEvaluator):
    def __init__(self, num_classes, year=2007):
        self.use_07_metric = year == 2007
        super().__init__(num_classes, ("bbox",))

    def evaluate(self):
        preds, gts = self._collect()
        return {"bbox": voc_evaluate(preds, gts, self.num_classes, self.use_07_metric)}


class CityscapesInstanceEvaluator(_InstanceEvaluator):
    """Cityscapes instance-level AP: mask AP over IoU 0.50:0.95 and AP50."""

    def __init__(self, num_classes):
        super().__init__(num_classes, ("segm",))

    def evaluate(self):
        preds, gts = self._collect()
        task = "segm" if all("masks" in p for p in preds) and all("masks" in g for g in gts) else "bbox"
        r = _summarize(instance_ap(preds, gts, self.num_classes, iou_type=task, max_dets=100,
                                   area_ranges={"all": AREA_RANGES["all"]}))
        return {task: {"AP": r["AP"], "AP50": r["AP50"]}}


class SemSegEvaluator(DatasetEvaluator):
    """``outputs[i]["sem_seg"]``: [K, H, W] scores (argmax taken) or [H, W]
    labels; ``inputs[i]["sem_seg"]``: [H, W] ground-truth labels."""

    def __init__(self, num_classes, ignore_label=255, class_names=None):
        self.num_classes = num_classes
        self.ignore_label = ignore_label
        self.class_names = class_names
        self.reset()

    def reset(self):
        self._conf = np.zeros((self.num_classes + 1, self.num_classes + 1), dtype=np.int64)

    def process(self, inputs, outputs):
        for x, o in zip(inputs, outputs):
            s = o["sem_seg"]
            pred = s.argmax(0) if s.dim() == 3 else s
            self._conf += semseg_confusion(_to_np(pred), _to_np(x["sem_seg"]), self.num_classes,
                                           self.ignore_label)

    def evaluate(self):
        conf = self._conf
        from ..parallel.dist import get_world_size
        if get_world_size() > 1:
            import torch.distributed as dist
            t = torch.from_numpy(conf)
            if dist.get_backend() == "nccl":  # RCCL: device tensors only
                t = t.to(torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(t)
            conf = t.cpu().numpy()
        return {"sem_seg": semseg_metrics(conf, self.class_names)}


class CityscapesSemSegEvaluator(SemSegEvaluator):
    """Cityscapes semantic segmentation on the 19 train ids (255 = ignore)."""

    def __init__(self, class_names=None):
        super().__init__(19, 255, class_names)


class DatasetEvaluators(DatasetEvaluator):
    def __init__(self, evaluators):
        self._evaluators = list(evaluators)

    def reset(self):
        for e in self._evaluators:
            e.reset()

    def process(self, inputs, outputs):
        for e in self._evaluators:
            e.process(inputs, outputs)

    def evaluate(self):
        res = {}
        for e in self._evaluators:
            for k, v in e.evaluate().items():
                if k in res:
                    raise KeyError(f"two evaluators produced {k!r}")
                res[k] = v
        return res


def build_evaluator(evaluator_type, num_classes, *, mask_on=False, sem_seg_classes=None,
                    ignore_label=255, category_frequency=None):
    """The reference's evaluator_type dispatch (``train_net.py:64-104``)."""
    tasks = ("bbox", "segm") if mask_on else ("bbox",)
    evs = []
    if evaluator_type in ("sem_seg", "coco_panoptic_seg"):
        evs.append(SemSegEvaluator(sem_seg_classes or num_classes, ignore_label))
    if evaluator_type in ("coco", "coco_panoptic_seg"):
        evs.append(COCOEvaluator(num_classes, tasks))
    if evaluator_type == "cityscapes_instance":
        return CityscapesInstanceEvaluator(num_classes)
    if evaluator_type == "cityscapes_sem_seg":
        return CityscapesSemSegEvaluator()
    if evaluator_type == "pascal_voc":
        return PascalVOCDetectionEvaluator(num_classes)
    if evaluator_type == "lvis":
        return LVISEvaluator(num_classes, tasks, category_frequency=category_frequency)
    if not evs:
        raise NotImplementedError(f"no evaluator for evaluator_type {evaluator_type!r}")
    return evs[0] if len(evs) == 1 else DatasetEvaluators(evs)


@torch.no_grad()
def inference_on_dataset(model, dataset, evaluator, num_images=None, autocast=None):
    """Run ``model`` over this rank's share of ``dataset`` and evaluate."""
    import contextlib
    from ..parallel.dist import get_rank, get_world_size
    autocast = autocast or contextlib.nullcontext
    was_training = model.training
    model.eval()
    evaluator.reset()
    n = len(dataset) if num_images is None else min(num_images, len(dataset))
    for i in range(get_rank(), n, get_world_size()):
        x = dataset[i]
        with autocast():
            out = model([x])
        evaluator.process([x], out)
    model.train(was_training)
    return evaluator.evaluate()
