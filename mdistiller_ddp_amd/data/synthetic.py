"""Synthetic data of a dataset's shape (there is no network for datasets).

Two flavours:

* :class:`SyntheticLoader` -- a small pool of ready, normalised batches kept
  on the device and replayed; what the benchmarks time (data cost excluded,
  like the reference's "training time" inset).
* :func:`synthetic_loaders` -- random uint8 images of the dataset's shape fed
  through the real device-resident pipeline (:class:`DeviceImageLoader`:
  shard sampler, on-device crop/flip/normalise kernel, CRD sampler), used by
  ``DATASET.SYNTHETIC`` so the trainer/CLI exercise every data-path piece.
"""
from __future__ import annotations

import numpy as np
import torch

from .cifar100 import CIFAR100_MEAN, CIFAR100_STD, DeviceImageLoader
from .common import CRDSampler

# name -> (C, H, W), num_classes, num_train, num_val
_SHAPES = {
    "cifar100": ((3, 32, 32), 100, 50000, 10000),
    "tiny_imagenet": ((3, 64, 64), 200, 100000, 10000),
    "imagenet": ((3, 224, 224), 1000, 1281167, 50000),
}

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
TINY_MEAN = (0.4802, 0.4481, 0.3975)
TINY_STD = (0.2302, 0.2265, 0.2262)
_NORM = {"cifar100": (CIFAR100_MEAN, CIFAR100_STD), "tiny_imagenet": (TINY_MEAN, TINY_STD),
         "imagenet": (IMAGENET_MEAN, IMAGENET_STD)}

# stored rows of a synthetic uint8 set (indices beyond wrap around): bounds host
# RAM on CPU runs while keeping num_data (the CRD memory size) the real one
_MAX_ROWS_BYTES = 256 << 20


def dataset_shape(name: str):
    """-> ((C, H, W), num_classes, num_train, num_val)."""
    if name not in _SHAPES:
        raise NotImplementedError(name)
    return _SHAPES[name]


class SyntheticLoader:
    """``steps_per_epoch`` batches cycling over ``pool`` pre-built device batches.

    Images are N(0, 1) (already "normalised"), labels uniform, ``index``
    uniform in ``[0, num_data)`` and, with ``crd_k``, ``contrastive_index``
    ``[B, K+1]`` whose column 0 is the sample's own index (CRD exact mode).
    """

    def __init__(self, dataset: str, batch_size: int, device, steps_per_epoch: int = 100,
                 pool: int = 4, seed: int = 0, crd_k: int = 0, num_data: int | None = None,
                 channels_last: bool = False, dtype=torch.float32):
        (c, h, w), ncls, ntrain, _ = dataset_shape(dataset)
        self.num_classes = ncls
        self.num_data = int(num_data or ntrain)
        self.steps_per_epoch = int(steps_per_epoch)
        dev = torch.device(device)
        g = torch.Generator().manual_seed(int(seed))
        self.batches = []
        for _ in range(max(1, min(int(pool), self.steps_per_epoch))):
            x = torch.randn(batch_size, c, h, w, generator=g).to(dtype)
            b = {"image": x.to(dev), "target": torch.randint(0, ncls, (batch_size,), generator=g).to(dev),
                 "index": torch.randint(0, self.num_data, (batch_size,), generator=g).to(dev)}
            if channels_last:
                b["image"] = b["image"].contiguous(memory_format=torch.channels_last)
            if crd_k:
                ci = torch.randint(0, self.num_data, (batch_size, int(crd_k) + 1), generator=g)
                ci[:, 0] = b["index"].cpu()
                b["contrastive_index"] = ci.to(dev)
            self.batches.append(b)

    def set_epoch(self, epoch: int) -> None:
        pass

    def __len__(self) -> int:
        return self.steps_per_epoch

    def __iter__(self):
        for i in range(self.steps_per_epoch):
            yield self.batches[i % len(self.batches)]


def synthetic_loaders(cfg, device, crd: bool):
    """(train, val, num_data) of random uint8 images through the device pipeline."""
    name = cfg.DATASET.TYPE
    (c, h, w), ncls, ntrain, nval = dataset_shape(name)
    n = int(cfg.DATASET.SYNTHETIC_SIZE) or ntrain
    nv = min(nval, n)
    rows = max(1, min(n, _MAX_ROWS_BYTES // (c * h * w)))
    rows_v = max(1, min(nv, _MAX_ROWS_BYTES // (c * h * w)))
    seed = max(int(cfg.EXPERIMENT.SEED), 0)
    rng = np.random.default_rng(seed + 17)
    mean, std = _NORM[name]
    # labels per stored row; dataset index i is row i % rows
    y_rows = rng.integers(0, ncls, rows)
    yva = rng.integers(0, ncls, rows_v)
    y_full = y_rows[np.arange(n) % rows]
    sampler = (CRDSampler(y_full, ncls, cfg.CRD.NCE.K, mode=cfg.CRD.MODE,
                          replace=name != "cifar100", seed=seed) if crd else None)
    xtr = rng.integers(0, 256, (rows, h, w, c), dtype=np.uint8)
    xva = rng.integers(0, 256, (rows_v, h, w, c), dtype=np.uint8)
    pad = 4 if name == "cifar100" else 0
    train = DeviceImageLoader(xtr, y_rows, cfg.SOLVER.BATCH_SIZE, device, train=True, mean=mean,
                              std=std, pad=pad, crd=sampler, seed=seed, num_data=n)
    val = DeviceImageLoader(xva, yva, cfg.DATASET.TEST.BATCH_SIZE, device, train=False,
                            mean=mean, std=std, num_data=nv)
    return train, val, n
