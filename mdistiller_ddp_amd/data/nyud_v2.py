"""NYUd-v2 depth dataset for the depth linear probe (reference
``dataset/nyud_v2.py:17-107``).

Reads ``<root>/nyud_v2.hdf5`` (``{train,test}/{images,depths}``), clips depth
to [0, 10] m and scales to [0, 1].  The reference's albumentations pipeline
(SmallestMaxSize(256) -> RandomResizedCrop(224, scale 0.8-1, ratio 1) ->
HFlip -> ColorJitter -> Normalize; test: SmallestMaxSize -> CenterCrop) is
reimplemented with PIL/numpy so image and depth receive the same geometric
transform.  ``h5py`` is required and imported lazily (it is not in this
image; the class raises a clear error without it).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch

MEAN = (0.485, 0.425, 0.385)
STD = (0.229, 0.224, 0.225)


def denormalize(x: torch.Tensor) -> torch.Tensor:
    """Undo the normalisation on a [3, H, W] or [B, 3, H, W] tensor (channel axis = the size-3 one)."""
    ch = [i for i, s in enumerate(x.shape) if s == 3][0]
    shape = [1] * x.ndim
    shape[ch] = 3
    m = torch.tensor(MEAN, dtype=x.dtype, device=x.device).view(shape)
    s = torch.tensor(STD, dtype=x.dtype, device=x.device).view(shape)
    return x * s + m


def _resize_pair(img, depth, size):
    from PIL import Image
    w, h = img.size
    sc = size / min(w, h)
    nw, nh = max(1, round(w * sc)), max(1, round(h * sc))
    return img.resize((nw, nh), Image.BILINEAR), depth.resize((nw, nh), Image.BILINEAR)


class NYUdTransform:
    def __init__(self, train: bool, img_size: int = 224, mean=MEAN, std=STD):
        self.train, self.size = train, img_size
        self.mean = np.asarray(mean, np.float32)
        self.std = np.asarray(std, np.float32)

    def __call__(self, image: np.ndarray, depth: np.ndarray):
        from PIL import Image, ImageEnhance
        img = Image.fromarray(np.ascontiguousarray(image).astype(np.uint8))
        dep = Image.fromarray(np.ascontiguousarray(depth).astype(np.float32), mode="F")
        img, dep = _resize_pair(img, dep, int(self.size * 256 / 224))
        w, h = img.size
        s = self.size
        if self.train:
            frac = random.uniform(0.8, 1.0)
            side = int(round(min(w, h) * np.sqrt(frac)))
            top, left = random.randint(0, h - side), random.randint(0, w - side)
            box = (left, top, left + side, top + side)
            img = img.resize((s, s), Image.BILINEAR, box=box)
            dep = dep.resize((s, s), Image.BILINEAR, box=box)
            if random.random() < 0.5:
                img, dep = img.transpose(Image.FLIP_LEFT_RIGHT), dep.transpose(Image.FLIP_LEFT_RIGHT)
            if random.random() < 0.5:
                img = ImageEnhance.Brightness(img).enhance(random.uniform(0.8, 1.2))
                img = ImageEnhance.Contrast(img).enhance(random.uniform(0.8, 1.2))
                img = ImageEnhance.Color(img).enhance(random.uniform(0.9, 1.1))
        else:
            top, left = (h - s) // 2, (w - s) // 2
            img = img.crop((left, top, left + s, top + s))
            dep = dep.crop((left, top, left + s, top + s))
        a = (np.asarray(img, np.float32) / 255.0 - self.mean) / self.std
        return torch.from_numpy(a.transpose(2, 0, 1).copy()), torch.from_numpy(np.asarray(dep, np.float32).copy())


class NYUdV2(torch.utils.data.Dataset):
    def __init__(self, dataroot: str, split: str = "train", transform=None):
        try:
            import h5py
        except ImportError as e:  # pragma: no cover - h5py is absent in this image
            raise ImportError("NYUdV2 needs h5py (not installed in this environment)") from e
        self.file = h5py.File(os.path.join(dataroot, "nyud_v2.hdf5"), "r")
        self.data = self.file.get(split)
        self.transform = transform or NYUdTransform(train=split == "train")

    def __len__(self):
        return len(self.data["images"])

    def __getitem__(self, index: int, return_masks: bool = False):
        image = self.data["images"][index]
        depth = np.clip(self.data["depths"][index], 0, 10) / 10.0
        image, depth = self.transform(image, depth)
        return (image, depth, depth > 0) if return_masks else (image, depth)
