"""Per-image detection containers on plain tensors.

The Detectron2 structures the reference's meta-architecture passes around
(`detection/model/rcnn.py:159-240`: ``ImageList``, ``Instances`` with
``gt_boxes`` / ``gt_classes`` / ``proposal_boxes`` ...) reduced to what the
RCNN stack here needs.  Boxes are ``[N, 4]`` float tensors (x1, y1, x2, y2)
in absolute pixels.
"""
from __future__ import annotations

import torch


class Instances:
    """Fields of equal length describing the objects of one image."""

    def __init__(self, image_size, **fields):
        object.__setattr__(self, "image_size", (int(image_size[0]), int(image_size[1])))
        object.__setattr__(self, "_fields", {})
        for k, v in fields.items():
            self.set(k, v)

    def set(self, name, value):
        if self._fields and len(value) != len(self):
            raise ValueError(f"field {name!r} has length {len(value)}, expected {len(self)}")
        self._fields[name] = value

    def has(self, name) -> bool:
        return name in self._fields

    def get(self, name):
        return self._fields[name]

    def remove(self, name):
        del self._fields[name]

    def get_fields(self) -> dict:
        return dict(self._fields)

    def __getattr__(self, name):
        fields = self.__dict__.get("_fields", {})
        if name in fields:
            return fields[name]
        raise AttributeError(f"Instances has no field {name!r}")

    def __setattr__(self, name, value):
        if name in ("image_size", "_fields"):
            object.__setattr__(self, name, value)
        else:
            self.set(name, value)

    def __len__(self) -> int:
        for v in self._fields.values():
            return len(v)
        return 0

    def __getitem__(self, item):
        if isinstance(item, int):
            item = slice(item, item + 1) if item != -1 else slice(-1, None)
        out = Instances(self.image_size)
        for k, v in self._fields.items():
            out.set(k, v[item])
        return out

    def to(self, device) -> "Instances":
        out = Instances(self.image_size)
        for k, v in self._fields.items():
            out.set(k, v.to(device) if hasattr(v, "to") else v)
        return out

    def __repr__(self):
        return (f"Instances(num={len(self)}, image_size={self.image_size}, "
                f"fields=[{', '.join(self._fields)}])")


class ImageList:
    """A padded batch of images plus the true (h, w) of each one."""

    def __init__(self, tensor: torch.Tensor, image_sizes):
        self.tensor = tensor
        self.image_sizes = [tuple(int(v) for v in s) for s in image_sizes]

    def __len__(self):
        return len(self.image_sizes)

    @staticmethod
    def from_tensors(tensors, size_divisibility: int = 0, pad_value: float = 0.0,
                     channels_last: bool = False) -> "ImageList":
        sizes = [(int(t.shape[-2]), int(t.shape[-1])) for t in tensors]
        H = max(s[0] for s in sizes)
        W = max(s[1] for s in sizes)
        if size_divisibility > 1:
            d = size_divisibility
            H, W = (H + d - 1) // d * d, (W + d - 1) // d * d
        c = tensors[0].shape[0]
        out = tensors[0].new_full((len(tensors), c, H, W), pad_value)
        for i, t in enumerate(tensors):
            out[i, :, :t.shape[-2], :t.shape[-1]].copy_(t)
        if channels_last:
            out = out.contiguous(memory_format=torch.channels_last)
        return ImageList(out, sizes)
