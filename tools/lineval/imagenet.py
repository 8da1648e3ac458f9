"""ImageNet linear probe of a trained student (reference `tools/lineval/imagenet.py`).

    python -m tools.lineval.imagenet <expname> -t best [-bs 512 -e 5 -lr 0.1]

Frozen backbone through the staged API (forward_stem -> get_layers ->
forward_pool); a new Linear(in_features, 1000) head trained with SGD +
per-iteration cosine annealing; log.yaml, best.pt / last.pt with the head.
Like the reference it expects a transformer student.
"""
from __future__ import annotations

import os
import sys
from argparse import ArgumentParser

import torch
from torch import optim
from torch.optim import lr_scheduler

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from tools.lineval.utils import init_parser, prepare_lineval_dir, load_from_checkpoint, frozen_features  # noqa: E402


def _loaders(args):
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.data import get_dataset
    cfg = get_cfg()
    cfg.DATASET.TYPE = "imagenet"
    cfg.DATASET.SYNTHETIC = bool(args.synthetic)
    cfg.DATASET.SYNTHETIC_SIZE = 4 * args.batch_size if args.synthetic else 0
    cfg.SOLVER.BATCH_SIZE = args.batch_size
    cfg.DATASET.TEST.BATCH_SIZE = args.test_batch_size
    cfg.DATASET.NUM_WORKERS = args.num_workers
    tr, te, _, _ = get_dataset(cfg, torch.device("cuda", args.device) if torch.cuda.is_available() else "cpu")
    return tr, te


def _xy(batch):
    if isinstance(batch, dict):
        return batch["image"], batch["target"]
    return batch[0], batch[1]


def main(argv=None, expected_arch="transformer"):
    parser = ArgumentParser("lineval.imagenet")
    init_parser(parser)
    args = parser.parse_args(argv)
    dev = torch.device("cuda", args.device) if torch.cuda.is_available() else torch.device("cpu")
    log_dir, log_file, best_file, last_file = prepare_lineval_dir(
        args.expname, tag=args.tag, dataset="imagenet", args=vars(args), root=args.output_root)
    train_loader, test_loader = _loaders(args)
    model, _ = load_from_checkpoint(args.expname, tag=args.tag, expected_arch=expected_arch,
                                    root=args.output_root)
    model = model.to(dev).eval()
    head = torch.nn.Linear(model.get_head().in_features, 1000).to(dev)
    opt = optim.SGD(head.parameters(), lr=args.learning_rate, momentum=args.momentum,
                    weight_decay=args.weight_decay)
    sched = lr_scheduler.CosineAnnealingLR(opt, T_max=args.epochs * len(train_loader), eta_min=1e-8)
    best = -1.0
    hist = {k: [] for k in ("train_loss", "train_top1", "test_loss", "test_top1")}
    for epoch in range(args.epochs):
        tot = torch.zeros(3, device=dev, dtype=torch.float64)
        for batch in train_loader:
            x, y = _xy(batch)
            x, y = x.to(dev).float(), y.to(dev)
            logit = head(frozen_features(model, x).float())
            loss = torch.nn.functional.cross_entropy(logit, y)
            loss.backward()
            opt.step()
            opt.zero_grad()
            sched.step()
            tot += torch.stack([loss.detach().double() * y.numel(),
                                (logit.argmax(1) == y).sum().double(), torch.tensor(y.numel(), device=dev, dtype=torch.float64)])
        tr = tot.tolist()
        ev = torch.zeros(3, device=dev, dtype=torch.float64)
        with torch.no_grad():
            for batch in test_loader:
                x, y = _xy(batch)
                x, y = x.to(dev).float(), y.to(dev)
                logit = head(frozen_features(model, x).float())
                ev += torch.stack([torch.nn.functional.cross_entropy(logit, y, reduction="sum").double(),
                                   (logit.argmax(1) == y).sum().double(), torch.tensor(y.numel(), device=dev, dtype=torch.float64)])
        te = ev.tolist()
        row = dict(train_loss=tr[0] / tr[2], train_top1=100 * tr[1] / tr[2],
                   test_loss=te[0] / te[2], test_top1=100 * te[1] / te[2])
        for k, v in row.items():
            hist[k].append(v)
        with open(log_file, "a") as f:
            print(f"- epoch: {epoch + 1}", file=f)
            for k, v in row.items():
                print(f"  {k}: {v:.4f}", file=f)
            print(file=f)
        ckpt = dict(epoch=epoch + 1, **hist, head={k: v.detach().cpu() for k, v in head.state_dict().items()})
        if row["test_top1"] > best:
            best = row["test_top1"]
            torch.save(ckpt, str(best_file))
        torch.save(ckpt, str(last_file))
    return best


if __name__ == "__main__":
    main()
