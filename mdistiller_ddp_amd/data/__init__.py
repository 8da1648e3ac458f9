"""Datasets: ``get_dataset(cfg, device) -> (train_loader, val_loader, num_data, num_classes)``.

Reference dispatcher: ``dataset/__init__.py:6-64`` (CIFAR-100 / ImageNet /
Tiny-ImageNet, CRD-sample variants when the distiller is CRD).  Here:

* ``DATASET.SYNTHETIC`` -- random uint8 images of the dataset's shape through
  the device-resident pipeline (no files needed; used by tests/benches).
* cifar100 -- device-resident set + HIP crop/flip/normalise kernel.
* imagenet / tiny_imagenet -- folder datasets decoded by CPU workers.

``cfg.SOLVER.BATCH_SIZE`` / ``cfg.DATASET.TEST.BATCH_SIZE`` are per-rank
batch sizes here (``tools/train.py`` divides the global ones by world size).
Train batches carry ``index`` (and ``contrastive_index`` for CRD trainers);
val batches are ``(image, target)``.
"""
from __future__ import annotations

from .common import CRDSampler, ShardSampler, make_loader
from .synthetic import SyntheticLoader, dataset_shape

NUM_CLASSES = {"cifar100": 100, "imagenet": 1000, "tiny_imagenet": 200}


def needs_crd(cfg) -> bool:
    return cfg.DISTILLER.TYPE in ("CRD", "CRDKD") or cfg.SOLVER.TRAINER in ("crd", "crd_dot")


def get_dataset(cfg, device="cpu"):
    import torch
    device = torch.device(device)
    typ = cfg.DATASET.TYPE
    if typ not in NUM_CLASSES:
        raise NotImplementedError(typ)
    crd = needs_crd(cfg)
    if cfg.DATASET.SYNTHETIC:
        from .synthetic import synthetic_loaders
        train, val, n = synthetic_loaders(cfg, device, crd)
    elif typ == "cifar100":
        from .cifar100 import get_cifar100_loaders
        train, val, n = get_cifar100_loaders(cfg, device, crd)
    else:
        from .imagefolder import get_folder_dataloaders
        train, val, n = get_folder_dataloaders(cfg, typ, crd)
    return train, val, n, NUM_CLASSES[typ]


__all__ = ["get_dataset", "NUM_CLASSES", "SyntheticLoader", "dataset_shape", "CRDSampler",
           "ShardSampler", "make_loader", "needs_crd"]
