#!/usr/bin/env python
"""Evaluate one model (reference `tools/eval.py`; same flags).

    python tools/eval.py -m resnet8x4 -c output/.../student_best -d cifar100 [-bs 64]
    python -m torch.distributed.run --nproc-per-node=8 tools/eval.py -m ResNet18 -c pretrain -d imagenet

Works with or without the launcher.  Under data parallelism every rank
evaluates its own un-padded shard and the counts are all-reduced (the
reference builds a non-sharded ImageNet loader inside a DDP group, so every
rank evaluates the full set and the metrics are duplicated).
``--synthetic`` evaluates on synthetic data of the dataset's shape.
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-m", "--model", type=str, default="")
    p.add_argument("-c", "--ckpt", type=str, default="pretrain")
    p.add_argument("-d", "--dataset", type=str, default="cifar100",
                   choices=["cifar100", "imagenet", "tiny_imagenet"])
    p.add_argument("-bs", "--batch-size", type=int, default=64)
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    args = p.parse_args(argv)

    import torch
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.data import get_dataset, NUM_CLASSES
    from mdistiller_ddp_amd.distillers import Vanilla
    from mdistiller_ddp_amd.engine.build import load_checkpoint
    from mdistiller_ddp_amd.engine.utils import validate
    from mdistiller_ddp_amd.engine.trainer import strip_module
    from mdistiller_ddp_amd.models import (cifar_model_dict, imagenet_model_dict,
                                           tiny_imagenet_model_dict)
    from mdistiller_ddp_amd.parallel import dist as D
    from mdistiller_ddp_amd.utils.logging import log_msg

    info = D.init_distributed()
    ws = info.world_size
    cfg = get_cfg()
    cfg.DATASET.TYPE = args.dataset
    cfg.DATASET.TEST.BATCH_SIZE = max(1, args.batch_size // ws)
    cfg.DATASET.SYNTHETIC = args.synthetic
    cfg.freeze()
    nc = NUM_CLASSES[args.dataset]
    if args.dataset == "imagenet":
        if args.ckpt == "pretrain":
            model = imagenet_model_dict[args.model](pretrained=True, num_classes=nc)
        else:
            model = imagenet_model_dict[args.model](pretrained=False, num_classes=nc)
            model.load_state_dict(strip_module(load_checkpoint(args.ckpt)["model"]))
    else:
        table = tiny_imagenet_model_dict if args.dataset == "tiny_imagenet" else cifar_model_dict
        ctor, pre = table[args.model]
        model = ctor(num_classes=nc)
        ckpt = pre if args.ckpt == "pretrain" else args.ckpt
        model.load_state_dict(strip_module(load_checkpoint(ckpt)["model"]))
    _, val_loader, _, _ = get_dataset(cfg, info.device)
    model = Vanilla(model).to(info.device)
    if info.device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    top1, top5, loss = validate(val_loader, model, info.device, dtype)
    if D.is_master():
        print(log_msg("Top-1:{:.3f}| Top-5:{:.3f}| Loss:{:.4f}".format(top1, top5, loss), "EVAL"))
    D.destroy()
    return top1, top5, loss


if __name__ == "__main__":
    main()
