"""Data pipeline on CPU: shard sampler, CRD sampler (native + numpy),
device-resident loader, synthetic get_dataset, CIFAR file parsing, folder
datasets and transforms."""
import numpy as np
import pytest
import torch

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.data import NUM_CLASSES, get_dataset
from mdistiller_ddp_amd.data.common import CRDSampler, ShardSampler


def test_shard_sampler_partitions_and_reshuffles():
    n, w = 103, 4
    parts = [ShardSampler(n, shuffle=True, seed=3, pad=True, rank=r, world=w) for r in range(w)]
    idx = np.concatenate([p.indices() for p in parts])
    assert len(idx) == 104 and set(idx.tolist()) == set(range(n))
    assert all(len(p) == 26 for p in parts)
    e0 = parts[0].indices().copy()
    parts[0].set_epoch(1)
    assert not np.array_equal(e0, parts[0].indices())  # D11: new shuffle per epoch
    ev = [ShardSampler(n, shuffle=False, pad=False, rank=r, world=w) for r in range(w)]
    assert sorted(np.concatenate([e.indices() for e in ev]).tolist()) == list(range(n))
    assert sum(len(e) for e in ev) == n


@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("mode,replace", [("exact", False), ("relax", False), ("exact", True)])
def test_crd_sampler(native, mode, replace, monkeypatch):
    from mdistiller_ddp_amd.ops import _ext
    if not native:
        monkeypatch.setattr(_ext, "available", lambda kind="hip": False)
    elif not _ext.available("host"):
        pytest.skip("host library not built")
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 10, 500)
    s = CRDSampler(labels, 10, 64, mode=mode, replace=replace, seed=1)
    index = rng.choice(500, 32, replace=False)
    out = s.sample(labels[index], index, seed=5)
    assert out.shape == (32, 65)
    if mode == "exact":
        assert np.array_equal(out[:, 0], index)
    else:
        assert np.array_equal(labels[out[:, 0]], labels[index])
    for b in range(32):
        neg = out[b, 1:]
        assert (labels[neg] != labels[index[b]]).all()
        assert ((neg >= 0) & (neg < 500)).all()
        if not replace:
            assert len(set(neg.tolist())) == 64
    assert np.array_equal(out, s.sample(labels[index], index, seed=5))  # deterministic per seed


def _cfg(typ="cifar100", crd=False, size=64):
    cfg = get_cfg()
    cfg.DATASET.TYPE = typ
    cfg.DATASET.SYNTHETIC = True
    cfg.DATASET.SYNTHETIC_SIZE = size
    cfg.SOLVER.BATCH_SIZE = 16
    cfg.DATASET.TEST.BATCH_SIZE = 16
    cfg.CRD.NCE.K = 8
    if crd:
        cfg.DISTILLER.TYPE = "CRD"
        cfg.SOLVER.TRAINER = "crd"
    return cfg


@pytest.mark.parametrize("typ", ["cifar100", "tiny_imagenet"])
def test_synthetic_get_dataset(typ):
    tr, va, n, nc = get_dataset(_cfg(typ, crd=True), "cpu")
    assert n == 64 and nc == NUM_CLASSES[typ]
    assert len(tr) == 4
    hw = 32 if typ == "cifar100" else 64
    seen = []
    for b in tr:
        assert b["image"].shape == (16, 3, hw, hw) and b["image"].dtype == torch.float32
        assert b["contrastive_index"].shape == (16, 9)
        assert torch.equal(b["contrastive_index"][:, 0], b["index"])
        seen.append(b["index"])
    assert sorted(torch.cat(seen).tolist()) == list(range(64))
    x, y = next(iter(va))
    assert x.shape[0] == 16 and y.shape == (16,)


def test_device_loader_eval_is_plain_normalise():
    from mdistiller_ddp_amd.data.cifar100 import CIFAR100_MEAN, CIFAR100_STD, DeviceImageLoader
    x = np.random.default_rng(0).integers(0, 256, (20, 32, 32, 3), dtype=np.uint8)
    ld = DeviceImageLoader(x, np.arange(20) % 7, 8, "cpu", train=False)
    img, tgt = next(iter(ld))
    ref = (torch.from_numpy(x[:8]).permute(0, 3, 1, 2).float() / 255
           - torch.tensor(CIFAR100_MEAN).view(1, 3, 1, 1)) / torch.tensor(CIFAR100_STD).view(1, 3, 1, 1)
    torch.testing.assert_close(img, ref)
    assert tgt.tolist() == [i % 7 for i in range(8)]


def test_augment_ref_crop_flip():
    from mdistiller_ddp_amd.data.cifar100 import augment_ref
    x = torch.arange(2 * 4 * 4 * 3, dtype=torch.uint8).view(2, 4, 4, 3)
    idx = torch.tensor([1])
    out = augment_ref(x, idx, torch.tensor([[2, 2]], dtype=torch.int32), torch.tensor([0], dtype=torch.uint8),
                      mean=(0, 0, 0), std=(1, 1, 1), pad=2)
    torch.testing.assert_close(out[0], x[1].permute(2, 0, 1).float() / 255)  # centred crop == identity
    out = augment_ref(x, idx, torch.tensor([[0, 0]], dtype=torch.int32), torch.tensor([1], dtype=torch.uint8),
                      mean=(0, 0, 0), std=(1, 1, 1), pad=2)
    shifted = torch.zeros(3, 4, 4)
    shifted[:, 2:, 2:] = x[1, :2, :2].permute(2, 0, 1).float() / 255
    torch.testing.assert_close(out[0], shifted.flip(2))


def test_cifar_binary_and_python_formats(tmp_path):
    import pickle
    from mdistiller_ddp_amd.data.cifar100 import load_cifar100
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (5, 3, 32, 32), dtype=np.uint8)
    fine = rng.integers(0, 100, 5)
    b = tmp_path / "b" / "cifar-100-binary"
    b.mkdir(parents=True)
    rec = np.concatenate([np.zeros((5, 1), np.uint8), fine.astype(np.uint8)[:, None], img.reshape(5, -1)], 1)
    rec.tofile(b / "train.bin")
    x, y = load_cifar100(str(tmp_path / "b"), True)
    assert np.array_equal(x, img.transpose(0, 2, 3, 1)) and np.array_equal(y, fine)
    p = tmp_path / "p" / "cifar-100-python"
    p.mkdir(parents=True)
    with open(p / "test", "wb") as f:
        pickle.dump({"data": img.reshape(5, -1), "fine_labels": fine.tolist()}, f)
    x, y = load_cifar100(str(tmp_path / "p"), False)
    assert np.array_equal(x, img.transpose(0, 2, 3, 1)) and np.array_equal(y, fine)
    with open(p / "train", "wb") as f:  # a pickle naming an arbitrary callable is refused
        pickle.dump({"data": print}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_cifar100(str(tmp_path / "p"), True)


def test_image_folder_and_crd_collate(tmp_path):
    from PIL import Image
    from mdistiller_ddp_amd.data.imagefolder import (CRDCollate, ImageFolderInstance,
                                                     imagenet_test_transform, imagenet_train_transform)
    for c in ("a", "b", "c"):
        (tmp_path / c).mkdir()
        for i in range(3):
            Image.fromarray(np.full((300, 260, 3), 40 * i, np.uint8)).save(tmp_path / c / f"{i}.png")
    ds = ImageFolderInstance(str(tmp_path), imagenet_train_transform())
    assert len(ds) == 9 and ds.classes == ["a", "b", "c"]
    img, t, i = ds[4]
    assert img.shape == (3, 224, 224) and t == 1 and i == 4
    ds_te = ImageFolderInstance(str(tmp_path), imagenet_test_transform(), with_index=False)
    assert ds_te[0][0].shape == (3, 224, 224)
    col = CRDCollate(CRDSampler(ds.targets, 3, 5, replace=True))
    x, tgt, idx, ci = col([ds[j] for j in (0, 4, 8)])
    assert x.shape == (3, 3, 224, 224) and ci.shape == (3, 6)
    assert (ds.targets[ci[:, 1:].numpy()] != tgt.numpy()[:, None]).all()
