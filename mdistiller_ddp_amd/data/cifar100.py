"""CIFAR-100 (and any small image set) as a device-resident loader.

Reference: ``dataset/cifar100.py`` -- ``CIFAR100Instance`` returns
``(img, target, index)`` (``:14-19``), ``CIFAR100InstanceSample`` adds the
CRD contrastive indices (``:23-113``), the train transform is
RandomCrop(32, pad 4) + HFlip + ToTensor + Normalize (``:116-126``), test is
ToTensor + Normalize (``:129-135``).

MI355X design: the whole train set is 50000 x 32 x 32 x 3 uint8 = 150 MB,
a rounding error in 288 GB of HBM.  It is uploaded once; each batch is a
gather + crop + flip + normalise done by one HIP kernel
(``ops/csrc/aug.hip::mda_crop_flip_norm``) that writes the NHWC
(channels-last) layout the conv kernels read, in bf16 or fp32.  No PIL, no
worker processes, no host->device image copies per step.  Batches are dicts
``{"image", "target", "index"[, "contrastive_index"]}`` (the trainer also
accepts the reference's tuples).

The CIFAR files are read without unpickling arbitrary objects: the binary
distribution (``cifar-100-binary/{train,test}.bin``) is parsed directly and
the python distribution (``cifar-100-python/{train,test}``) goes through a
restricted unpickler that only admits numpy array reconstruction.
"""
from __future__ import annotations

import io
import math
import os
import pickle

import numpy as np
import torch

from .common import CRDSampler, ShardSampler, data_root

CIFAR100_MEAN = (0.5071, 0.4867, 0.4408)
CIFAR100_STD = (0.2675, 0.2565, 0.2761)


# ----------------------------------------------------------------------------
# file formats
class _NumpyOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar"), ("_codecs", "encode")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")


def _load_python_split(path):
    with open(path, "rb") as f:
        d = _NumpyOnlyUnpickler(io.BytesIO(f.read()), encoding="latin1").load()
    x = np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(x), np.asarray(d["fine_labels"], dtype=np.int64)


def _load_binary_split(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 2 + 3072)
    x = raw[:, 2:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(x), raw[:, 1].astype(np.int64)


def load_cifar100(root: str, train: bool):
    """-> (uint8 [N, 32, 32, 3] NHWC, int64 [N]) from ``root``."""
    split = "train" if train else "test"
    cands = [(os.path.join(root, "cifar-100-binary", split + ".bin"), _load_binary_split),
             (os.path.join(root, "cifar-100-python", split), _load_python_split)]
    for path, fn in cands:
        if os.path.exists(path):
            return fn(path)
    raise FileNotFoundError(
        f"CIFAR-100 not found under {root} (expected cifar-100-binary/ or cifar-100-python/); "
        "there is no download in this framework -- place the files there or set DATASET.SYNTHETIC")


# ----------------------------------------------------------------------------
# augmentation
def augment_ref(x: torch.Tensor, idx: torch.Tensor, offs: torch.Tensor, flip: torch.Tensor,
                mean=CIFAR100_MEAN, std=CIFAR100_STD, pad: int = 4) -> torch.Tensor:
    """PyTorch reference of the aug kernel: float32 NCHW.

    ``x`` uint8 [N, H, W, C]; ``offs`` [B, 2] crop offsets in [0, 2*pad] of
    the zero-padded image; ``flip`` [B] horizontal flip flags.
    """
    img = x[idx.long()].permute(0, 3, 1, 2).float() / 255.0
    b, c, h, w = img.shape
    if pad:
        img = torch.nn.functional.pad(img, (pad, pad, pad, pad))
    dev = img.device
    rows = offs[:, 0].long().view(b, 1) + torch.arange(h, device=dev).view(1, h)
    cols = offs[:, 1].long().view(b, 1) + torch.arange(w, device=dev).view(1, w)
    img = img.gather(2, rows.view(b, 1, h, 1).expand(b, c, h, img.shape[3]))
    img = img.gather(3, cols.view(b, 1, 1, w).expand(b, c, h, w))
    f = flip.bool().view(b, 1, 1, 1)
    img = torch.where(f, img.flip(3), img)
    m = torch.tensor(mean, device=dev).view(1, c, 1, 1)
    s = torch.tensor(std, device=dev).view(1, c, 1, 1)
    return (img - m) / s


class DeviceImageLoader:
    """Device-resident image set with on-device augmentation.

    ``x`` uint8 [N, H, W, C] (numpy or tensor), ``y`` int labels.  ``train``
    enables the random crop (zero padding ``pad``) and horizontal flip; the
    eval path is a plain normalise.  Shards by rank with an epoch-seeded
    shuffle (:class:`ShardSampler`); ``index_map`` maps dataset indices to
    stored rows (synthetic sets store fewer rows than they index).
    """

    def __init__(self, x, y, batch_size: int, device, train: bool = True, out_dtype=torch.float32,
                 mean=CIFAR100_MEAN, std=CIFAR100_STD, pad: int = 4, shuffle=None,
                 drop_last: bool = False, crd: CRDSampler | None = None, seed: int = 0,
                 num_data: int | None = None, channels_last: bool = True):
        self.device = torch.device(device)
        self.x = torch.as_tensor(x).to(self.device)
        assert self.x.dtype == torch.uint8 and self.x.dim() == 4, "x must be uint8 [N, H, W, C]"
        self.y_host = np.asarray(y, dtype=np.int64)
        self.y = torch.as_tensor(self.y_host).to(self.device)
        self.n = int(num_data if num_data is not None else len(self.y_host))
        self.rows = self.x.shape[0]
        self.batch_size = int(batch_size)
        self.train = train
        self.out_dtype = out_dtype
        self.pad = pad if train else 0
        self.drop_last = drop_last
        self.crd = crd
        self.channels_last = channels_last
        c = self.x.shape[3]
        self.mean = torch.tensor(mean[:c], dtype=torch.float32, device=self.device)
        self.inv_std = 1.0 / torch.tensor(std[:c], dtype=torch.float32, device=self.device)
        self._mean, self._std = tuple(mean[:c]), tuple(std[:c])
        self.sampler = ShardSampler(self.n, shuffle=train if shuffle is None else shuffle,
                                    seed=seed, pad=train)
        self.seed = int(seed)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(self._epoch_seed(0))
        self.epoch = 0

    def _epoch_seed(self, epoch: int) -> int:
        # a function of (seed, epoch, rank) only: a resumed run replays the
        # exact augmentation stream of an uninterrupted one
        return (self.seed * 1000003 + int(epoch) * 7919 + self.sampler.rank * 104729) & 0x7FFFFFFF

    # the trainer calls this every epoch
    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)
        self.sampler.set_epoch(epoch)

    def __len__(self) -> int:
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _rows(self, idx: torch.Tensor) -> torch.Tensor:
        return idx if self.rows == self.n else torch.remainder(idx, self.rows)

    def _make(self, idx: torch.Tensor) -> torch.Tensor:
        """Augmented, normalised images for dataset rows ``idx`` (device int64)."""
        b = idx.shape[0]
        _, h, w, c = self.x.shape
        if self.pad:
            offs = torch.randint(0, 2 * self.pad + 1, (b, 2), generator=self.gen, device=self.device,
                                 dtype=torch.int32)
            flip = torch.randint(0, 2, (b,), generator=self.gen, device=self.device, dtype=torch.uint8)
        elif self.train:
            offs = torch.zeros(b, 2, dtype=torch.int32, device=self.device)
            flip = torch.randint(0, 2, (b,), generator=self.gen, device=self.device, dtype=torch.uint8)
        else:
            offs = torch.zeros(b, 2, dtype=torch.int32, device=self.device)
            flip = torch.zeros(b, dtype=torch.uint8, device=self.device)
        from ..ops.backend import hip_enabled_for
        if hip_enabled_for(self.x) and self.out_dtype in (torch.float32, torch.bfloat16):
            from ..ops import _ext
            out = torch.empty(b, h, w, c, dtype=self.out_dtype, device=self.device)
            _ext.call("mda_crop_flip_norm", self.x, idx.contiguous(), offs, flip, self.mean,
                      self.inv_std, out, 0 if self.out_dtype == torch.float32 else 1, b, h, w, c,
                      self.pad)
            img = out.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
            return img if self.channels_last else img.contiguous()
        img = augment_ref(self.x, idx, offs, flip, self._mean, self._std, self.pad).to(self.out_dtype)
        return img.contiguous(memory_format=torch.channels_last) if self.channels_last else img

    def __iter__(self):
        order = self.sampler.indices()
        self.gen.manual_seed(self._epoch_seed(self.epoch))
        bs = self.batch_size
        nb = len(self)
        for i in range(nb):
            ids = order[i * bs:(i + 1) * bs]
            idx_host = torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int64))
            idx = idx_host.to(self.device, non_blocking=True)
            rows = self._rows(idx)
            batch = {"image": self._make(rows), "target": self.y[rows]}
            if self.train:
                batch["index"] = idx
            if self.crd is not None:
                tgt = self.y_host[ids % len(self.y_host)]
                ci = self.crd.sample(tgt, ids, seed=(self.epoch * 1000003 + i) * 131 + self.sampler.rank)
                batch["contrastive_index"] = torch.from_numpy(ci).to(self.device, non_blocking=True)
            if self.train:
                yield batch
            else:
                yield batch["image"], batch["target"]


def get_cifar100_loaders(cfg, device, crd: bool):
    root = data_root(cfg)
    xtr, ytr = load_cifar100(root, True)
    xte, yte = load_cifar100(root, False)
    dt = torch.float32
    sampler = (CRDSampler(ytr, 100, cfg.CRD.NCE.K, mode=cfg.CRD.MODE, replace=False,
                          seed=cfg.EXPERIMENT.SEED if cfg.EXPERIMENT.SEED >= 0 else 0)
               if crd else None)
    train = DeviceImageLoader(xtr, ytr, cfg.SOLVER.BATCH_SIZE, device, train=True, out_dtype=dt,
                              crd=sampler, seed=max(cfg.EXPERIMENT.SEED, 0))
    val = DeviceImageLoader(xte, yte, cfg.DATASET.TEST.BATCH_SIZE, device, train=False, out_dtype=dt)
    return train, val, len(ytr)
