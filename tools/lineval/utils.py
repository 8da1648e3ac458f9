"""Linear-probe helpers (reference `tools/lineval/utils.py:10-98`).

Experiments are looked up under ``output/<exp_name>`` (``--output-root`` to
change): ``code/_cfg.yaml`` (safe YAML) and ``student_<tag>`` (loaded with
``weights_only=True``).
"""
from __future__ import annotations

import os
from argparse import ArgumentParser
from datetime import datetime
from pathlib import Path

import torch

OUTPUT_ROOT = os.environ.get("MDA_OUTPUT_ROOT", "output")


def get_config(exp_name: str, ckpt_tag=None, root: str = None):
    from mdistiller_ddp_amd.config import load_cfg
    exp_root = os.path.join(root or OUTPUT_ROOT, exp_name)
    with open(os.path.join(exp_root, "code", "_cfg.yaml")) as f:
        cfg = load_cfg(f)
    if ckpt_tag is None:
        return cfg
    ckpt = torch.load(os.path.join(exp_root, f"student_{ckpt_tag}"), map_location="cpu",
                      weights_only=True)
    return cfg, ckpt


def prepare_lineval_dir(exp_name: str, tag="latest", dataset: str = "imagenet", args: dict = None,
                        root: str = None):
    lineval_dir = Path(root or OUTPUT_ROOT).joinpath(exp_name, "lineval")
    nowstr = datetime.now().strftime("_%y%m%d_%H%M%S")
    log_dir = lineval_dir.joinpath(str(tag), dataset + nowstr)
    log_dir.mkdir(parents=True)
    if args is not None:
        with open(log_dir.joinpath("_cfg.yaml"), "w") as f:
            for k, v in args.items():
                print(f"{k}: {v}", file=f)
    return (log_dir, log_dir.joinpath("log.yaml"), log_dir.joinpath("best.pt"),
            log_dir.joinpath("last.pt"))


def load_from_checkpoint(exp_name: str, tag="latest", expected_arch=None, root: str = None):
    from mdistiller_ddp_amd.models.imagenet import imagenet_model_dict
    cfg, ckpt = get_config(exp_name, ckpt_tag=tag, root=root)
    model = imagenet_model_dict[cfg.DISTILLER.STUDENT](pretrained=False)
    if expected_arch is not None and model.get_arch() != expected_arch:
        raise ValueError(f"Expected {expected_arch}, but this checkpoint requires {model.get_arch()}.")
    result = model.load_state_dict(ckpt["model"], strict=False)
    return model, result


def T_CHECKPOINT_TAG(tag: str):
    if tag in {"latest", "best"}:
        return tag
    if tag.isdigit():
        return int(tag)
    raise ValueError(tag)


def init_parser(parser: ArgumentParser, defaults: dict = None) -> ArgumentParser:
    parser.add_argument("expname", type=str)
    parser.add_argument("--tag", "-t", type=T_CHECKPOINT_TAG, default="best")
    parser.add_argument("--device", "-d", type=int, default=0)
    parser.add_argument("--batch-size", "-bs", type=int, default=512)
    parser.add_argument("--test-batch-size", "-tbs", type=int, default=512)
    parser.add_argument("--num-workers", "-nw", type=int, default=8)
    parser.add_argument("--epochs", "-e", type=int, default=5)
    parser.add_argument("--learning-rate", "-lr", type=float, default=0.1)
    parser.add_argument("--momentum", type=float, default=0.9)
    parser.add_argument("--weight-decay", type=float, default=1.0e-6)
    parser.add_argument("--output-root", type=str, default=None)
    parser.add_argument("--synthetic", action="store_true",
                        help="synthetic data of the dataset's shape (no dataset on disk)")
    parser.set_defaults(**(defaults or {}))
    return parser


def frozen_features(model, x):
    """Staged forward of a frozen backbone: stem -> layers -> pool."""
    with torch.no_grad():
        y = model.forward_stem(x)
        for layer in model.get_layers():
            y = layer(model.activate(y)) if model.get_arch() == "cnn" else layer(y)
        return model.forward_pool(y)
