"""Detection training loop + evaluator (the reference drives Detectron2's
``DefaultTrainer`` / ``SimpleTrainer`` / ``COCOEvaluator``,
`detection/train_net.py:46-172`).

* Student parameters (everything outside ``teacher.*`` that requires grad,
  incl. the ReviewKD ABF chain) live in one flat fp32 buffer
  (:class:`..engine.optim.FlatParams`): one fused SGD launch per step and
  bucketed RCCL all-reduce of gradient slices overlapped with backward
  (:class:`..parallel.grad_reducer.GradReducer`) -- no DDP wrapper, the
  frozen teacher never touches the wire.
* ``WarmupMultiStepLR`` (linear warm-up, step decay at ``SOLVER.STEPS``).
* bf16 autocast on the GPU (``RUNTIME.DTYPE``); losses are fp32.
* Checkpoints: ``model`` (student + teacher state dict), ``optimizer``
  (torch-format SGD state), ``iteration``; ``resume`` restarts after the
  last saved iteration (Detectron2 ``resume_or_load`` semantics).
* :func:`coco_evaluate`: COCO bbox AP (AP, AP50, AP75, APs/m/l; 101-point
  interpolated precision, 10 IoU thresholds, maxDets 100) computed in numpy
  -- pycocotools is not installed in this image.
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import numpy as np
import torch

from ..engine.optim import FlatParams, FlatSGD
from ..parallel.dist import get_rank, get_world_size, is_master
from ..parallel.grad_reducer import GradReducer
from .boxes import pairwise_iou


def warmup_multistep_lr(it, base_lr, steps, gamma, warmup_iters, warmup_factor, method="linear"):
    f = 1.0
    if it < warmup_iters:
        if method == "constant":
            f = warmup_factor
        else:
            a = it / warmup_iters
            f = warmup_factor * (1 - a) + a
    return base_lr * f * gamma ** sum(1 for s in steps if it >= s)


class DetectionTrainer:
    def __init__(self, cfg, model, loader, device, log=print):
        self.cfg = cfg
        self.model = model
        self.loader = loader
        self.device = device
        self.log = log
        params = model.student_parameters() if hasattr(model, "student_parameters") else \
            [p for p in model.parameters() if p.requires_grad]
        self.flat = FlatParams(params)
        s = cfg.SOLVER
        world = get_world_size()
        self.opt = FlatSGD(self.flat, s.BASE_LR, momentum=s.MOMENTUM, weight_decay=s.WEIGHT_DECAY,
                           grad_clip=(s.CLIP_GRADIENTS.CLIP_VALUE if s.CLIP_GRADIENTS.ENABLED
                                      and s.CLIP_GRADIENTS.CLIP_TYPE == "norm" else 0.0),
                           grad_scale=1.0 / world)
        self.reducer = GradReducer(self.flat, bucket_mb=float(cfg.RUNTIME.BUCKET_MB))
        self.iter = 0
        self.use_bf16 = device.type == "cuda" and cfg.RUNTIME.DTYPE == "bf16"

    def lr_at(self, it):
        s = self.cfg.SOLVER
        return warmup_multistep_lr(it, s.BASE_LR, s.STEPS, s.GAMMA, s.WARMUP_ITERS, s.WARMUP_FACTOR,
                                   s.WARMUP_METHOD)

    def autocast(self):
        if self.use_bf16:
            return torch.autocast("cuda", dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def run_step(self, batch):
        self.opt.set_lr(self.lr_at(self.iter))
        self.flat.zero_grad()
        with self.autocast():
            losses = self.model(batch)
        total = sum(losses.values())
        self.reducer.arm()
        total.backward()
        self.reducer.finish()
        self.opt.step()
        self.iter += 1
        return total, losses

    def train(self, max_iter=None, start_iter=0, ckpt_dir=None):
        cfg = self.cfg
        max_iter = int(max_iter or cfg.SOLVER.MAX_ITER)
        self.iter = start_iter
        self.model.train()
        it = iter(self.loader)
        t0 = time.time()
        period = int(cfg.RUNTIME.LOG_PERIOD)
        while self.iter < max_iter:
            total, losses = self.run_step(next(it))
            if (self.iter % period == 0 or self.iter == max_iter) and is_master():
                vals = {k: float(v.detach()) for k, v in losses.items()}
                if not np.isfinite(sum(vals.values())):
                    raise FloatingPointError(f"loss became non-finite at iter {self.iter}: {vals}")
                dt = (time.time() - t0) / period
                t0 = time.time()
                self.log(f"iter {self.iter}/{max_iter} lr {self.opt.lr:.5f} total {sum(vals.values()):.4f} "
                         + " ".join(f"{k} {v:.4f}" for k, v in vals.items()) + f" | {dt * 1e3:.1f} ms/it")
            if ckpt_dir and (self.iter % int(cfg.SOLVER.CHECKPOINT_PERIOD) == 0 or self.iter == max_iter):
                self.save(ckpt_dir)

    # checkpointing ---------------------------------------------------------
    def save(self, ckpt_dir, name=None):
        if not is_master():
            return
        os.makedirs(ckpt_dir, exist_ok=True)
        obj = {"model": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
               "optimizer": self.opt.state_dict(), "iteration": self.iter}
        path = os.path.join(ckpt_dir, name or f"model_{self.iter - 1:07d}.pth")
        torch.save(obj, path + ".tmp")
        os.replace(path + ".tmp", path)
        with open(os.path.join(ckpt_dir, "last_checkpoint"), "w") as f:
            f.write(os.path.basename(path))

    def resume(self, ckpt_dir) -> int:
        marker = os.path.join(ckpt_dir, "last_checkpoint")
        if not os.path.exists(marker):
            return 0
        with open(marker) as f:
            path = os.path.join(ckpt_dir, f.read().strip())
        obj = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(obj["model"])
        self.opt.load_state_dict(obj["optimizer"])
        self.iter = int(obj["iteration"])
        return self.iter


# ----------------------------------------------------------------------------- evaluation
def _ap_101(tp, conf, n_gt):
    if n_gt == 0:
        return None
    if len(tp) == 0:
        return 0.0
    order = np.argsort(-conf, kind="mergesort")
    tp = tp[order]
    ctp = np.cumsum(tp)
    cfp = np.cumsum(1 - tp)
    rec = ctp / n_gt
    prec = ctp / np.maximum(ctp + cfp, np.spacing(1))
    prec = np.maximum.accumulate(prec[::-1])[::-1]
    rs = np.linspace(0, 1, 101)
    idx = np.searchsorted(rec, rs, side="left")
    q = np.where(idx < len(prec), prec[np.minimum(idx, len(prec) - 1)], 0.0)
    return float(q.mean())


AREA_RANGES = {"all": (0, 1e10), "small": (0, 32 ** 2), "medium": (32 ** 2, 96 ** 2), "large": (96 ** 2, 1e10)}


def coco_evaluate(predictions, ground_truths, num_classes, max_dets=100):
    """``predictions`` / ``ground_truths``: per image dicts with numpy
    ``boxes`` [N, 4] (xyxy), ``classes`` [N] and (pred) ``scores`` [N].
    Greedy COCO matching per (image, class, IoU threshold, area range)."""
    ious = np.linspace(0.5, 0.95, 10)
    res = {}
    for area_name, (lo, hi) in AREA_RANGES.items():
        aps = np.full((len(ious), num_classes), np.nan)
        for c in range(num_classes):
            tps = [[] for _ in ious]
            n_gt = 0
            for p, g in zip(predictions, ground_truths):
                gm = g["classes"] == c
                gb = g["boxes"][gm]
                ga = (gb[:, 2] - gb[:, 0]) * (gb[:, 3] - gb[:, 1])
                gign = (ga < lo) | (ga >= hi)
                n_gt += int((~gign).sum())
                pm = p["classes"] == c
                pb, ps = p["boxes"][pm], p["scores"][pm]
                o = np.argsort(-ps, kind="mergesort")[:max_dets]
                pb, ps = pb[o], ps[o]
                if len(pb) == 0:
                    continue
                iou = (pairwise_iou(torch.from_numpy(pb).float(), torch.from_numpy(gb).float()).numpy()
                       if len(gb) else np.zeros((len(pb), 0)))
                pa = (pb[:, 2] - pb[:, 0]) * (pb[:, 3] - pb[:, 1])
                gorder = np.argsort(gign, kind="mergesort")  # non-ignored gts first
                for ti, t in enumerate(ious):
                    used = np.zeros(len(gb), bool)
                    tp = np.zeros(len(pb))
                    ign = np.zeros(len(pb), bool)
                    for d in range(len(pb)):
                        best, m = min(t, 1 - 1e-10), -1
                        for gi in gorder:
                            if used[gi]:
                                continue
                            if m > -1 and not gign[m] and gign[gi]:
                                break
                            if iou[d, gi] < best:
                                continue
                            best, m = iou[d, gi], gi
                        if m >= 0:
                            used[m] = True
                            ign[d] = gign[m]
                            tp[d] = 1.0
                        else:
                            ign[d] = pa[d] < lo or pa[d] >= hi
                    keep = ~ign
                    tps[ti].append((tp[keep], ps[keep]))
            for ti in range(len(ious)):
                tp_all = np.concatenate([a for a, _ in tps[ti]]) if tps[ti] else np.zeros(0)
                cf_all = np.concatenate([b for _, b in tps[ti]]) if tps[ti] else np.zeros(0)
                ap = _ap_101(tp_all, cf_all, n_gt)
                if ap is not None:
                    aps[ti, c] = ap
        with np.errstate(all="ignore"):
            per_t = np.nanmean(aps, axis=1) if np.isfinite(aps).any() else np.full(len(ious), np.nan)
        if area_name == "all":
            res["AP"] = float(np.nanmean(per_t) * 100)
            res["AP50"] = float(per_t[0] * 100)
            res["AP75"] = float(per_t[5] * 100)
        else:
            res["AP" + area_name[0]] = float(np.nanmean(per_t) * 100) if np.isfinite(per_t).any() else float("nan")
    return res


@torch.no_grad()
def run_inference(model, dataset, num_images, device, autocast=contextlib.nullcontext):
    model.eval()
    preds, gts = [], []
    rank, world = get_rank(), get_world_size()
    for i in range(rank, min(num_images, len(dataset)), world):
        x = dataset[i]
        with autocast():
            out = model([x])[0]["instances"]
        sy = x["height"] / x["instances"].image_size[0]
        sx = x["width"] / x["instances"].image_size[1]
        g = x["instances"].gt_boxes.float().cpu().numpy() * np.array([sx, sy, sx, sy])
        preds.append({"boxes": out.pred_boxes.float().cpu().numpy(), "scores": out.scores.float().cpu().numpy(),
                      "classes": out.pred_classes.cpu().numpy()})
        gts.append({"boxes": g, "classes": x["instances"].gt_classes.cpu().numpy()})
    if world > 1:
        import torch.distributed as dist
        allp = [None] * world
        allg = [None] * world
        dist.all_gather_object(allp, preds)
        dist.all_gather_object(allg, gts)
        preds = [p for r in allp for p in r]
        gts = [g for r in allg for g in r]
    model.train()
    return preds, gts


def dump_json(obj, path):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1)
