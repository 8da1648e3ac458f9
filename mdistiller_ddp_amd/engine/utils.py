"""Engine utilities (reference `mdistiller/engine/utils.py:12-146`):
meters, top-k accuracy, LR schedules, validation, checkpoint I/O.

Differences from the reference, all deliberate:

* ``adjust_learning_rate`` takes the actual iterations per epoch of this
  rank's loader, so the per-batch cosine schedule is right for any dataset
  and any world size (the reference divides the dataset size by the
  already-per-rank batch, running the schedule world_size x too slowly, and
  only knows two datasets -- SURVEY D12);
* ``validate`` keeps correct/total counts on the device and all-reduces
  three scalars per evaluation instead of all-gathering logits every batch,
  and uses an un-padded shard per rank, so no sample is counted twice;
* ``save_checkpoint`` is atomic (write to ``.tmp`` then rename), so a crash
  while writing never leaves a truncated ``latest``;
* ``load_checkpoint`` uses ``weights_only=True`` (no arbitrary unpickling).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from ..utils.logging import log_msg  # noqa: F401  (reference API)


class AverageMeter:
    """Computes and stores the average and current value."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def accuracy(output, target, topk=(1,)):
    with torch.no_grad():
        maxk = min(max(topk), output.shape[1])
        batch_size = target.size(0)
        _, pred = output.topk(maxk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.reshape(1, -1).expand_as(pred))
        return [correct[:k].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / batch_size)
                for k in topk]


def adjust_learning_rate(epoch: int, bidx: int, cfg, iters_per_epoch: int) -> float:
    """LR for (1-based) ``epoch`` and batch ``bidx`` of that epoch."""
    sch = cfg.SOLVER.SCHEDULE.TYPE
    base = cfg.SOLVER.LR
    if sch == "MULTISTEP":
        steps = int(np.sum(epoch > np.asarray(cfg.SOLVER.SCHEDULE.MULTISTEP.STAGES)))
        return base * (cfg.SOLVER.SCHEDULE.MULTISTEP.RATE ** steps)
    if sch == "COSINE":
        warm = cfg.SOLVER.SCHEDULE.COSINE.WARMUP
        nb = max(1, int(iters_per_epoch))
        n_warm = nb * warm
        g = (epoch - 1) * nb + bidx
        if g < n_warm:
            return base / n_warm * (g + 1)
        n_cos = max(1, nb * (cfg.SOLVER.EPOCHS - warm))
        last = base * cfg.SOLVER.SCHEDULE.COSINE.RATE
        return (math.cos((g - n_warm) / n_cos * math.pi) + 1.0) * 0.5 * (base - last) + last
    raise NotImplementedError(sch)


@torch.no_grad()
def validate(val_loader, distiller, device=None, dtype=None):
    """Global top-1 / top-5 / CE over the (rank-sharded) validation set."""
    from ..parallel import dist_fn
    from ..parallel.dist import is_master
    from .step import topk_rank
    from ..ops.nn import fp32_head
    distiller.eval()
    if device is None:
        device = next(distiller.parameters()).device
    acc = torch.zeros(4, dtype=torch.float64, device=device)  # loss_sum, top1, top5, n
    amp = (device.type == "cuda" and dtype in (torch.bfloat16, torch.float16))
    pbar = None
    if is_master() and hasattr(val_loader, "__len__"):
        try:
            from tqdm import tqdm
            pbar = tqdm(total=len(val_loader), dynamic_ncols=True, leave=False)
        except Exception:  # pragma: no cover
            pbar = None
    for image, target in val_loader:
        image = image.to(device, non_blocking=True).float()
        if device.type == "cuda":
            image = image.contiguous(memory_format=torch.channels_last)
        target = target.to(device, non_blocking=True)
        with torch.autocast("cuda", dtype=dtype, enabled=amp), fp32_head():
            out = distiller(image=image)
        out = out.float()
        rank = topk_rank(out, target)
        acc[0] += F.cross_entropy(out, target, reduction="sum").double()
        acc[1] += (rank < 1).sum().double()
        acc[2] += (rank < 5).sum().double()
        acc[3] += target.numel()
        if pbar is not None:
            pbar.update()
    if pbar is not None:
        pbar.close()
    acc = dist_fn.reduce(acc, "sum").cpu()
    n = max(acc[3].item(), 1.0)
    return 100.0 * acc[1].item() / n, 100.0 * acc[2].item() / n, acc[0].item() / n


def save_checkpoint(obj, path: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        torch.save(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def load_checkpoint(path: str):
    with open(path, "rb") as f:
        return torch.load(f, map_location="cpu", weights_only=True)
