"""Shared pieces of the visualisation tools (reference
``tools/visualizations/{tsne,correlation}.ipynb``, rewritten as scripts).

``collect`` runs a model over the validation split once and returns the
logits, the pooled features and the labels as numpy arrays; models are
loaded from the framework's checkpoint format (``{"model": state_dict}``,
``module.``-prefixed or not) with ``weights_only`` loading.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def val_loader(dataset: str, batch_size: int, synthetic: bool, device):
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.data import get_dataset
    cfg = get_cfg()
    cfg.DATASET.TYPE = dataset
    cfg.DATASET.TEST.BATCH_SIZE = batch_size
    cfg.DATASET.SYNTHETIC = synthetic
    cfg.freeze()
    _, loader, _, ncls = get_dataset(cfg, device)
    return loader, ncls


def load_model(dataset: str, name: str, ckpt: str, num_classes: int):
    """ckpt: path, "pretrain" (the zoo's teacher checkpoint) or "random"."""
    from mdistiller_ddp_amd.engine.build import load_checkpoint
    from mdistiller_ddp_amd.engine.trainer import strip_module
    from mdistiller_ddp_amd.models import build_model, teacher_ckpt_path
    model = build_model(dataset, name, num_classes)
    if ckpt == "pretrain":
        ckpt = teacher_ckpt_path(dataset, name)
    if ckpt and ckpt != "random":
        model.load_state_dict(strip_module(load_checkpoint(ckpt)["model"]))
    return model


def collect(model, loader, device, max_batches: int = 0):
    """(logits [n, C], pooled features [n, D], labels [n]) over the loader."""
    import torch
    model = model.to(device).eval()
    logits, feats, labels = [], [], []
    with torch.no_grad():
        for i, (image, target) in enumerate(loader):
            if max_batches and i >= max_batches:
                break
            out, f = model(image.to(device).float())
            logits.append(out.float().cpu().numpy())
            feats.append(f["pooled_feat"].float().reshape(out.shape[0], -1).cpu().numpy())
            labels.append(target.cpu().numpy())
    return np.concatenate(logits), np.concatenate(feats), np.concatenate(labels)


def save_figure(fig, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    fig.savefig(path, dpi=150, bbox_inches="tight")


def base_parser(description: str):
    import argparse
    p = argparse.ArgumentParser(description=description)
    p.add_argument("-d", "--dataset", default="cifar100",
                   choices=["cifar100", "tiny_imagenet", "imagenet"])
    p.add_argument("-bs", "--batch-size", type=int, default=256)
    p.add_argument("--synthetic", action="store_true",
                   help="synthetic validation data of the dataset's shape")
    p.add_argument("--max-batches", type=int, default=0, help="0 = whole split")
    p.add_argument("--device", default="cuda")
    p.add_argument("-o", "--out", default="output/visualizations")
    return p
