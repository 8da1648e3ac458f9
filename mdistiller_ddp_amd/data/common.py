"""Data-pipeline plumbing shared by every dataset.

* :class:`ShardSampler` -- the rank-strided epoch shuffle of the reference's
  ``DistributedSampler`` (``dataset/_common.py:5-11``), but with
  ``set_epoch`` actually honoured by the trainer and an
  unpadded mode for evaluation so no sample is counted twice.
* :func:`make_loader` -- the reference's loader factory signature
  ``make_loader(dataset, batch_size, num_workers, shuffle, use_ddp)``.  The
  worker count is *per rank* (the reference divides the global count by the
  world size and ends up with 0 workers at world >= 3).
* :class:`CRDSampler` -- CRD contrastive index sampling for a whole batch
  (reference ``cifar100.py:83-113``, ``imagenet.py:18-67``,
  ``tiny_imagenet.py:23-71``).  The reference builds a per-class list of all
  negatives (C x N int arrays, 1.28 G entries for ImageNet) and calls
  ``np.random.choice`` per sample inside the loader workers; here the
  samples are kept sorted by class once and the K negatives of a batch are
  drawn in native code (``ops/csrc/host/sampler.cpp``, OpenMP over the
  batch) by rank in the "not my class" index space.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))


def data_root(cfg=None) -> str:
    root = getattr(getattr(cfg, "DATASET", None), "ROOT", "") if cfg is not None else ""
    return root or os.environ.get("MDA_DATA_ROOT", os.path.join(REPO, "data"))


def _world():
    from ..parallel import dist as D
    return D.get_rank(), D.get_world_size()


class ShardSampler(torch.utils.data.Sampler):
    """Rank-strided, epoch-seeded shuffle.

    ``pad=True`` (training) repeats the head of the permutation so every rank
    sees the same number of samples, like ``DistributedSampler``;
    ``pad=False`` (evaluation) gives each sample to exactly one rank.
    """

    def __init__(self, n: int, shuffle: bool = True, seed: int = 0, pad: bool = True,
                 rank: int | None = None, world: int | None = None):
        r, w = _world()
        self.n = int(n)
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.shuffle = shuffle
        self.seed = seed
        self.pad = pad
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def indices(self) -> np.ndarray:
        if self.shuffle:
            g = np.random.default_rng((self.seed, self.epoch))
            perm = g.permutation(self.n)
        else:
            perm = np.arange(self.n)
        if self.pad and self.world > 1:
            total = math.ceil(self.n / self.world) * self.world
            if total > self.n:
                perm = np.concatenate([perm, perm[: total - self.n]])
        return perm[self.rank :: self.world]

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        if self.pad:
            return math.ceil(self.n / self.world)
        return len(range(self.rank, self.n, self.world))


def make_loader(dataset, batch_size: int, num_workers: int, shuffle: bool, use_ddp: bool,
                collate_fn=None, drop_last: bool = False):
    """``DataLoader`` over a map-style dataset; ``use_ddp`` shards by rank."""
    kw = dict(batch_size=batch_size, num_workers=num_workers, pin_memory=torch.cuda.is_available(),
              collate_fn=collate_fn, drop_last=drop_last,
              persistent_workers=num_workers > 0)
    if use_ddp:
        sampler = ShardSampler(len(dataset), shuffle=shuffle, pad=shuffle)
        return torch.utils.data.DataLoader(dataset, sampler=sampler, **kw)
    return torch.utils.data.DataLoader(dataset, shuffle=shuffle, **kw)


class CRDSampler:
    """Batch-wise CRD contrastive indices: ``[B, K+1]`` = positive + K negatives.

    mode ``exact``: the positive is the sample itself; ``relax``: a random
    sample of the same class.  Negatives come uniformly from the other
    classes, without replacement when ``K`` fits (the reference CIFAR
    behaviour) or with replacement (``replace=True``, the reference
    ImageNet/Tiny behaviour).
    """

    def __init__(self, labels, num_classes: int, k: int, mode: str = "exact",
                 replace: bool = False, seed: int = 0):
        if mode not in ("exact", "relax"):
            raise NotImplementedError(mode)
        labels = np.asarray(labels, dtype=np.int64)
        self.n = len(labels)
        self.k = int(k)
        self.mode = mode
        self.replace = replace
        self.seed = int(seed)
        self.labels = labels
        order = np.argsort(labels, kind="stable").astype(np.int64)
        count = np.bincount(labels, minlength=num_classes).astype(np.int64)
        start = np.concatenate([[0], np.cumsum(count)[:-1]]).astype(np.int64)
        self.cls_sorted, self.cls_count, self.cls_start = order, count, start
        self._calls = 0

    def sample(self, target, index, seed: int | None = None) -> np.ndarray:
        target = np.ascontiguousarray(np.asarray(target, dtype=np.int64))
        index = np.ascontiguousarray(np.asarray(index, dtype=np.int64))
        b = len(index)
        if seed is None:
            seed = self.seed * 1000003 + self._calls
            self._calls += 1
        out = np.empty((b, self.k + 1), dtype=np.int64)
        flags = (1 if self.replace else 0) | (2 if self.mode == "relax" else 0)
        from ..ops import _ext
        if _ext.available("host"):
            _ext.host_call("mdah_crd_sample", self.cls_sorted.ctypes.data, self.cls_start.ctypes.data,
                           self.cls_count.ctypes.data, target.ctypes.data, index.ctypes.data,
                           out.ctypes.data, b, self.k, self.n, flags, int(seed))
            return out
        return self._sample_np(target, index, out, int(seed))

    def _sample_np(self, target, index, out, seed):
        rng = np.random.default_rng(seed)
        for i in range(len(index)):
            c = target[i]
            st, cnt = self.cls_start[c], self.cls_count[c]
            nneg = self.n - cnt
            out[i, 0] = index[i] if self.mode == "exact" else self.cls_sorted[st + rng.integers(cnt)]
            if self.replace or self.k > nneg:
                r = rng.integers(0, nneg, self.k)
            else:
                r = rng.choice(nneg, self.k, replace=False)
            out[i, 1:] = np.where(r < st, self.cls_sorted[np.minimum(r, self.n - 1)],
                                  self.cls_sorted[np.minimum(r + cnt, self.n - 1)])
        return out
