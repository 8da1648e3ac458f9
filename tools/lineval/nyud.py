"""NYUd-v2 depth linear probe of a ViT student (reference `tools/lineval/nyud.py`).

    python -m tools.lineval.nyud <expname> -t best [-e 1000]

Patch tokens of the frozen ViT -> Linear(embed_dim, 256) -> each patch's
256 outputs become a 16x16 depth patch (einops rearrange) -> 224x224 depth
map; MSE loss, RMSE metric.  Requires ``h5py`` (and the reference's
``nyud_v2.hdf5``).  The best checkpoint is the LOWEST test RMSE (the
reference compares the wrong way round).
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

from tools.lineval.utils import init_parser, prepare_lineval_dir, load_from_checkpoint  # noqa: E402


def patches_to_depth(x: torch.Tensor) -> torch.Tensor:
    import einops
    _, num_patches, embed_dim = x.shape
    pr = int(num_patches ** 0.5)
    px = int(embed_dim ** 0.5)
    return einops.rearrange(x[:, -pr * pr:], "b (ph pw) (h w) -> b (ph h) (pw w)", ph=pr, pw=pr,
                            h=px, w=px)


def main(argv=None):
    from mdistiller_ddp_amd.data.nyud_v2 import NYUdV2
    from mdistiller_ddp_amd.data.common import make_loader
    parser = ArgumentParser("lineval.nyud")
    init_parser(parser, defaults=dict(epochs=1000))
    parser.add_argument("--dataroot", default=os.path.join(ROOT, "data", "nyud"))
    args = parser.parse_args(argv)
    dev = torch.device("cuda", args.device) if torch.cuda.is_available() else torch.device("cpu")
    log_dir, log_file, best_file, last_file = prepare_lineval_dir(
        args.expname, tag=args.tag, dataset="nyud", args=vars(args), root=args.output_root)
    train_loader = make_loader(NYUdV2(args.dataroot, "train"), args.batch_size, args.num_workers, True, True)
    test_loader = make_loader(NYUdV2(args.dataroot, "test"), args.test_batch_size, args.num_workers, False, False)
    model, _ = load_from_checkpoint(args.expname, tag=args.tag, root=args.output_root)
    model = model.to(dev).eval()
    head = torch.nn.Linear(model.embed_dim, 256).to(dev)
    opt = optim.SGD(head.parameters(), lr=args.learning_rate, weight_decay=args.weight_decay)
    sched = lr_scheduler.CosineAnnealingLR(opt, T_max=args.epochs * len(train_loader), eta_min=1e-8)
    best_rmse = float("inf")
    for epoch in range(args.epochs):
        for x, depth in train_loader:
            with torch.no_grad():
                t = model.forward_stem(x.to(dev))
                for blk in model.get_layers():
                    t = blk(t)
            pred = patches_to_depth(head(t))
            loss = torch.nn.functional.mse_loss(pred, depth.to(dev))
            loss.backward()
            opt.step()
            opt.zero_grad()
            sched.step()
        se, n = 0.0, 0
        with torch.no_grad():
            for x, depth in test_loader:
                t = model.forward_stem(x.to(dev))
                for blk in model.get_layers():
                    t = blk(t)
                pred = patches_to_depth(head(t))
                se += torch.nn.functional.mse_loss(pred, depth.to(dev), reduction="sum").item()
                n += depth.numel()
        rmse = (se / max(n, 1)) ** 0.5
        with open(log_file, "a") as f:
            print(f"- epoch: {epoch + 1}\n  test_rmse: {rmse:.4f}\n", file=f)
        ckpt = dict(epoch=epoch + 1, test_rmse=rmse, head={k: v.cpu() for k, v in head.state_dict().items()})
        if rmse < best_rmse:
            best_rmse = rmse
            torch.save(ckpt, str(best_file))
        torch.save(ckpt, str(last_file))
    return best_rmse


if __name__ == "__main__":
    main()
