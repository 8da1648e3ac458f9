"""Detection data: Detectron2-style ``batched_inputs`` (list of dicts with
``image`` [3, H, W] uint8/float, ``instances`` with ``gt_boxes`` /
``gt_classes`` / optional ``gt_masks``, ``height`` / ``width``).

* :class:`SyntheticDetection` -- COCO-shaped synthetic images and boxes
  (shortest edge drawn from ``INPUT.MIN_SIZE_TRAIN``, capped by
  ``MAX_SIZE_TRAIN``), the stand-in for ``coco_2017_train`` in this
  network-less image.  Images are generated ON THE DEVICE.
* :class:`COCODetection` -- a COCO-format instances json + image folder
  (PIL decode, shortest-edge resize, horizontal flip; masks rasterised from
  polygons with PIL) -- the ``DatasetMapper`` path of the reference's
  `detection/train_net.py` for users who have the files.
* :class:`DetectionLoader` -- per-rank sharded, infinite iterator of
  batches of ``IMS_PER_BATCH // world`` images (Detectron2's
  ``TrainingSampler`` semantics: every rank sees a disjoint stream).
"""
from __future__ import annotations

import json
import os
import random

import numpy as np
import torch

from .structures import Instances


def resize_shape(h, w, short, max_size):
    scale = short / min(h, w)
    if max(h, w) * scale > max_size:
        scale = max_size / max(h, w)
    return int(round(h * scale)), int(round(w * scale)), scale


class SyntheticDetection:
    def __init__(self, cfg, device="cpu", train=True, seed=0, num_images=1 << 30):
        self.min_sizes = list(cfg.INPUT.MIN_SIZE_TRAIN if train else (cfg.INPUT.MIN_SIZE_TEST,))
        self.max_size = int(cfg.INPUT.MAX_SIZE_TRAIN if train else cfg.INPUT.MAX_SIZE_TEST)
        self.fixed = tuple(int(v) for v in cfg.RUNTIME.SYNTHETIC_SIZE)
        self.num_classes = int(cfg.MODEL.ROI_HEADS.NUM_CLASSES)
        self.mask_on = bool(cfg.MODEL.MASK_ON)
        self.device = torch.device(device)
        self.seed = seed
        self.num_images = num_images

    def __len__(self):
        return self.num_images

    def __getitem__(self, i):
        rng = random.Random(self.seed * 1000003 + i)
        if self.fixed[0] > 0:
            H, W = self.fixed
        else:
            # COCO-like aspect ratios (4:3 landscape / portrait)
            h0, w0 = (480, 640) if rng.random() < 0.7 else (640, 480)
            H, W, _ = resize_shape(h0, w0, rng.choice(self.min_sizes), self.max_size)
        g = torch.Generator(device="cpu").manual_seed(self.seed * 7919 + i)
        n = rng.randint(1, 12)
        wh = torch.rand(n, 2, generator=g) * torch.tensor([W * 0.5, H * 0.5]) + 16
        xy = torch.rand(n, 2, generator=g) * (torch.tensor([W, H]) - wh).clamp(min=1)
        boxes = torch.cat([xy, xy + wh], 1)
        classes = torch.randint(0, self.num_classes, (n,), generator=g)
        if self.device.type == "cpu":
            img = torch.randint(0, 256, (3, H, W), dtype=torch.uint8, generator=g)
        else:  # generated where it is consumed: no host->device image copy per step
            img = torch.randint(0, 256, (3, H, W), dtype=torch.uint8, device=self.device)
        inst = Instances((H, W), gt_boxes=boxes.to(self.device), gt_classes=classes.to(self.device))
        if self.mask_on:
            ys = torch.arange(H).view(1, H, 1).float()
            xs = torch.arange(W).view(1, 1, W).float()
            cx, cy = (boxes[:, 0] + boxes[:, 2]) / 2, (boxes[:, 1] + boxes[:, 3]) / 2
            rx, ry = (boxes[:, 2] - boxes[:, 0]) / 2, (boxes[:, 3] - boxes[:, 1]) / 2
            m = (((xs - cx.view(-1, 1, 1)) / rx.view(-1, 1, 1)) ** 2
                 + ((ys - cy.view(-1, 1, 1)) / ry.view(-1, 1, 1)) ** 2) <= 1.0  # ellipses in boxes
            inst.set("gt_masks", m.to(torch.uint8).to(self.device))
        return {"image": img, "instances": inst, "height": H, "width": W, "image_id": i}


class COCODetection:
    """COCO-format json + images; category ids are mapped to contiguous 0..K-1."""

    def __init__(self, json_file, image_root, cfg, train=True, device="cpu"):
        with open(json_file) as f:
            d = json.load(f)
        cats = sorted(c["id"] for c in d["categories"])
        self.cat_map = {c: i for i, c in enumerate(cats)}
        self.inv_cat_map = {i: c for c, i in self.cat_map.items()}
        anns = {}
        for a in d.get("annotations", []):
            if a.get("iscrowd", 0):
                continue
            anns.setdefault(a["image_id"], []).append(a)
        self.images = [im for im in d["images"] if (not train) or im["id"] in anns]
        self.anns = anns
        self.root = image_root
        self.train = train
        self.min_sizes = list(cfg.INPUT.MIN_SIZE_TRAIN if train else (cfg.INPUT.MIN_SIZE_TEST,))
        self.max_size = int(cfg.INPUT.MAX_SIZE_TRAIN if train else cfg.INPUT.MAX_SIZE_TEST)
        self.flip = train and cfg.INPUT.RANDOM_FLIP == "horizontal"
        self.rgb = cfg.INPUT.FORMAT == "RGB"
        self.mask_on = bool(cfg.MODEL.MASK_ON)
        self.device = torch.device(device)

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        from PIL import Image, ImageDraw
        info = self.images[i]
        im = Image.open(os.path.join(self.root, info["file_name"])).convert("RGB")
        w0, h0 = im.size
        H, W, s = resize_shape(h0, w0, random.choice(self.min_sizes), self.max_size)
        im = im.resize((W, H), Image.BILINEAR)
        arr = np.asarray(im)
        if not self.rgb:
            arr = arr[:, :, ::-1]
        flip = self.flip and random.random() < 0.5
        if flip:
            arr = arr[:, ::-1]
        img = torch.from_numpy(np.ascontiguousarray(arr.transpose(2, 0, 1)))
        boxes, classes, masks = [], [], []
        for a in self.anns.get(info["id"], []):
            x, y, bw, bh = a["bbox"]
            if bw < 1 or bh < 1:
                continue
            b = [x * s, y * s, (x + bw) * s, (y + bh) * s]
            if flip:
                b = [W - b[2], b[1], W - b[0], b[3]]
            boxes.append(b)
            classes.append(self.cat_map[a["category_id"]])
            if self.mask_on:
                m = Image.new("L", (W, H), 0)
                for poly in a.get("segmentation", []) if isinstance(a.get("segmentation"), list) else []:
                    pts = [(px * s, py * s) for px, py in zip(poly[0::2], poly[1::2])]
                    if flip:
                        pts = [(W - px, py) for px, py in pts]
                    if len(pts) >= 3:
                        ImageDraw.Draw(m).polygon(pts, fill=1)
                masks.append(torch.from_numpy(np.asarray(m, dtype=np.uint8).copy()))
        inst = Instances((H, W), gt_boxes=torch.tensor(boxes, dtype=torch.float32).reshape(-1, 4),
                         gt_classes=torch.tensor(classes, dtype=torch.int64))
        if self.mask_on:
            inst.set("gt_masks", torch.stack(masks) if masks else torch.zeros((0, H, W), dtype=torch.uint8))
        return {"image": img, "instances": inst, "height": h0, "width": w0, "image_id": info["id"]}


class DetectionLoader:
    """Infinite per-rank iterator over a dataset (disjoint strided shards)."""

    def __init__(self, dataset, images_per_rank, rank=0, world=1, shuffle=True, seed=0):
        self.ds = dataset
        self.bs = int(images_per_rank)
        self.rank, self.world = rank, world
        self.shuffle = shuffle
        self.seed = seed
        self._epoch = 0

    def _indices(self):
        n = len(self.ds)
        if n > (1 << 24):  # virtual synthetic set: a fresh strided range per epoch
            base = self._epoch * (1 << 20)
            return range(base + self.rank, base + (1 << 20), self.world)
        g = torch.Generator().manual_seed(self.seed + self._epoch)
        order = torch.randperm(n, generator=g).tolist() if self.shuffle else list(range(n))
        return order[self.rank::self.world]

    def __iter__(self):
        while True:
            batch = []
            for i in self._indices():
                batch.append(self.ds[i])
                if len(batch) == self.bs:
                    yield batch
                    batch = []
            self._epoch += 1


def build_detection_data(cfg, rank=0, world=1, train=True, device="cpu"):
    rt = cfg.RUNTIME
    if rt.COCO_JSON:
        ds = COCODetection(rt.COCO_JSON, rt.COCO_IMAGE_ROOT, cfg, train=train)
    else:
        ds = SyntheticDetection(cfg, device=device, train=train, seed=rank if train else 10_000,
                                num_images=(1 << 30) if train else int(rt.SYNTHETIC_VAL_IMAGES))
    ims = max(1, int(cfg.SOLVER.IMS_PER_BATCH) // max(world, 1))
    return ds, DetectionLoader(ds, ims if train else 1, rank, world, shuffle=train)


def category_info(ds):
    return getattr(ds, "inv_cat_map", None)

