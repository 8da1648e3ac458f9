"""ImageNet and Tiny-ImageNet from class-per-directory folders.

Reference: ``dataset/imagenet.py`` (``ImageNet(ImageFolder)`` with index
``:12-15``, ``ImageNetInstanceSample`` ``:18-67``, RandomResizedCrop(224) +
HFlip / Resize(256) + CenterCrop(224) ``:69-91``, val loader ``:110-118``) and
``dataset/tiny_imagenet.py`` (RandomRotation(20) + HFlip ``:74-115``).

torchvision is not part of this stack, so folder scanning, PIL decoding and
the geometric transforms are implemented here (PIL + numpy) with
torchvision's sampling rules (RandomResizedCrop: 10 tries of scale
[0.08, 1] / log-uniform ratio [3/4, 4/3], centre-crop fallback; bilinear
resize).  Decoding stays on CPU workers; the normalise step is fused into a
single uint8 -> float conversion.  CRD negatives are drawn per batch in
native code (:class:`~.common.CRDSampler`) inside the collate function
instead of per sample with the C x N negative tables of the reference.
"""
from __future__ import annotations

import math
import os
import random

import numpy as np
import torch

from .common import CRDSampler, data_root, make_loader
from .synthetic import IMAGENET_MEAN, IMAGENET_STD, TINY_MEAN, TINY_STD

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def scan_folder(root: str):
    """-> (samples [(path, class_idx)], classes) for ``root/<class>/<image>``."""
    classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
    if not classes:
        raise FileNotFoundError(f"no class folders under {root}")
    samples = []
    for ci, c in enumerate(classes):
        for dirpath, _, files in sorted(os.walk(os.path.join(root, c), followlinks=True)):
            for f in sorted(files):
                if f.lower().endswith(IMG_EXTENSIONS):
                    samples.append((os.path.join(dirpath, f), ci))
    return samples, classes


def _pil():
    from PIL import Image
    return Image


# ----------------------------------------------------------------------------
# transforms (PIL in, PIL out; ToTensorNormalize last)
class RandomResizedCrop:
    def __init__(self, size, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3)):
        self.size, self.scale, self.ratio = size, scale, ratio

    def params(self, w, h):
        area = w * h
        lr = (math.log(self.ratio[0]), math.log(self.ratio[1]))
        for _ in range(10):
            ta = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(*lr))
            cw = int(round(math.sqrt(ta * ar)))
            ch = int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                return random.randint(0, h - ch), random.randint(0, w - cw), ch, cw
        r = w / h
        if r < self.ratio[0]:
            cw, ch = w, int(round(w / self.ratio[0]))
        elif r > self.ratio[1]:
            ch, cw = h, int(round(h * self.ratio[1]))
        else:
            cw, ch = w, h
        return (h - ch) // 2, (w - cw) // 2, ch, cw

    def __call__(self, img):
        top, left, ch, cw = self.params(*img.size)
        return img.resize((self.size, self.size), _pil().BILINEAR, box=(left, top, left + cw, top + ch))


class RandomHorizontalFlip:
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, img):
        return img.transpose(_pil().FLIP_LEFT_RIGHT) if random.random() < self.p else img


class Resize:
    """Resize the shorter side to ``size`` (torchvision int semantics)."""

    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        w, h = img.size
        if w <= h:
            nw, nh = self.size, int(self.size * h / w)
        else:
            nh, nw = self.size, int(self.size * w / h)
        return img.resize((nw, nh), _pil().BILINEAR)


class CenterCrop:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        w, h = img.size
        top = int(round((h - self.size) / 2.0))
        left = int(round((w - self.size) / 2.0))
        return img.crop((left, top, left + self.size, top + self.size))


class RandomRotation:
    def __init__(self, degrees):
        self.degrees = degrees

    def __call__(self, img):
        return img.rotate(random.uniform(-self.degrees, self.degrees), _pil().NEAREST, expand=False,
                          fillcolor=0)


class ToTensorNormalize:
    def __init__(self, mean, std):
        self.mean = np.asarray(mean, np.float32).reshape(3, 1, 1)
        self.inv = 1.0 / np.asarray(std, np.float32).reshape(3, 1, 1)

    def __call__(self, img):
        a = np.asarray(img.convert("RGB"), dtype=np.float32).transpose(2, 0, 1) * (1.0 / 255.0)
        return torch.from_numpy((a - self.mean) * self.inv)


class Compose:
    def __init__(self, ts):
        self.ts = ts

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


def imagenet_train_transform(mean=IMAGENET_MEAN, std=IMAGENET_STD):
    return Compose([RandomResizedCrop(224), RandomHorizontalFlip(), ToTensorNormalize(mean, std)])


def imagenet_test_transform(mean=IMAGENET_MEAN, std=IMAGENET_STD):
    return Compose([Resize(256), CenterCrop(224), ToTensorNormalize(mean, std)])


def tiny_train_transform():
    return Compose([RandomRotation(20), RandomHorizontalFlip(0.5), ToTensorNormalize(TINY_MEAN, TINY_STD)])


def tiny_test_transform():
    return Compose([ToTensorNormalize(TINY_MEAN, TINY_STD)])


# ----------------------------------------------------------------------------
class ImageFolderInstance(torch.utils.data.Dataset):
    """``(img, target, index)`` per sample (``with_index``) or ``(img, target)``."""

    def __init__(self, root: str, transform=None, with_index: bool = True):
        self.root = root
        self.samples, self.classes = scan_folder(root)
        self.targets = np.asarray([t for _, t in self.samples], dtype=np.int64)
        self.transform = transform
        self.with_index = with_index

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, index):
        path, target = self.samples[index]
        with open(path, "rb") as f:
            img = _pil().open(f).convert("RGB")
        if self.transform is not None:
            img = self.transform(img)
        return (img, target, index) if self.with_index else (img, target)


class CRDCollate:
    """Batch collate that appends ``[B, K+1]`` contrastive indices."""

    def __init__(self, sampler: CRDSampler):
        self.sampler = sampler

    def __call__(self, items):
        img = torch.stack([it[0] for it in items])
        tgt = torch.as_tensor([it[1] for it in items], dtype=torch.int64)
        idx = torch.as_tensor([it[2] for it in items], dtype=torch.int64)
        seed = int.from_bytes(os.urandom(4), "little")
        ci = torch.from_numpy(self.sampler.sample(tgt.numpy(), idx.numpy(), seed=seed))
        return img, tgt, idx, ci


def get_folder_dataloaders(cfg, kind: str, crd: bool):
    """ImageNet (``kind='imagenet'``, ``<root>/imagenet/{train,val}``) or Tiny
    (``kind='tiny_imagenet'``, ``<root>/tiny-imagenet-200/{train,val}``)."""
    root = data_root(cfg)
    sub = "imagenet" if kind == "imagenet" else "tiny-imagenet-200"
    if kind == "imagenet":
        ttr, tte, nval_workers = imagenet_train_transform(), imagenet_test_transform(), 16
    else:
        ttr, tte, nval_workers = tiny_train_transform(), tiny_test_transform(), 1
    train_set = ImageFolderInstance(os.path.join(root, sub, "train"), ttr, with_index=True)
    test_set = ImageFolderInstance(os.path.join(root, sub, "val"), tte, with_index=False)
    use_ddp = bool(cfg.EXPERIMENT.DDP)
    collate = None
    if crd:
        collate = CRDCollate(CRDSampler(train_set.targets, len(train_set.classes), cfg.CRD.NCE.K,
                                        mode="exact", replace=True))
    nw = int(cfg.DATASET.NUM_WORKERS)
    train = make_loader(train_set, cfg.SOLVER.BATCH_SIZE, nw, True, use_ddp, collate_fn=collate)
    val = make_loader(test_set, cfg.DATASET.TEST.BATCH_SIZE, min(nw, nval_workers) if nw else 0,
                      False, use_ddp)
    return train, val, len(train_set)
