#!/usr/bin/env python
"""Training entry point (reference `tools/train.py`; same CLI).

    python -m torch.distributed.run --nproc-per-node=8 --master-addr 127.0.0.1 \
        tools/train.py --cfg configs/cifar100/dkd/res32x4_res8x4.yaml [more.yaml ...] \
        [--resume | --auto-resume] [KEY VALUE ...]

Also runs as a single process without the launcher.  One process per GPU;
RANK (global) / LOCAL_RANK (device) / WORLD_SIZE come from the launcher
(the reference treats LOCAL_RANK as the global rank).  As in the
reference, ``SOLVER.BATCH_SIZE`` and ``DATASET.TEST.BATCH_SIZE`` are global
and are divided by the world size (global-batch semantics of the published
hyper-parameters).
"""
from __future__ import annotations

import argparse
import os

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see mdistiller_ddp_amd/__init__.py
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def experiment_name_of(cfg, opts):
    name = cfg.EXPERIMENT.NAME or cfg.EXPERIMENT.TAG
    tags = cfg.EXPERIMENT.TAG.split(",")
    if opts:
        extra = ["{}:{}".format(k, str(v).replace(os.sep, "_")) for k, v in zip(opts[::2], opts[1::2])]
        tags += extra
        name += ",".join(extra)
    if len(name) > 160:  # keep the directory name within filesystem limits
        import hashlib
        name = name[:140] + "-" + hashlib.sha1(name.encode()).hexdigest()[:12]
    return os.path.join(cfg.EXPERIMENT.PROJECT, name), tags


def main(cfg, resume, opts, info):
    import torch
    from mdistiller_ddp_amd.config import dump_cfg
    from mdistiller_ddp_amd.data import get_dataset
    from mdistiller_ddp_amd.engine import trainer_dict, build_distiller
    from mdistiller_ddp_amd.parallel.dist import is_master
    from mdistiller_ddp_amd.utils.logging import log_msg

    experiment_name, tags = experiment_name_of(cfg, opts)
    if is_master() and cfg.LOG.WANDB:
        try:
            import wandb
            wandb.init(project=cfg.EXPERIMENT.PROJECT, name=experiment_name, tags=tags)
        except Exception:
            print(log_msg("Failed to use WANDB", "INFO"))
            cfg.defrost()
            cfg.LOG.WANDB = False
            cfg.freeze()
    if is_master():
        dump_cfg(cfg, show=True)
    train_loader, val_loader, num_data, num_classes = get_dataset(cfg, info.device)
    if is_master() and cfg.DISTILLER.TYPE != "NONE":
        print(log_msg("Loading teacher model", "INFO"), flush=True)
    distiller = build_distiller(cfg, num_classes, info.device, num_data)
    if cfg.DISTILLER.TYPE != "NONE" and is_master():
        print(log_msg("Extra parameters of {}: {:,d}".format(
            cfg.DISTILLER.TYPE, distiller.get_extra_parameters()), "INFO"), flush=True)
    trainer = trainer_dict[cfg.SOLVER.TRAINER](experiment_name, distiller, train_loader,
                                               val_loader, cfg, device=info.device)
    if resume == "auto":
        resume = os.path.exists(os.path.join(trainer.log_path, "latest"))
    trainer.train(resume=bool(resume))
    return trainer


def parse(argv=None):
    p = argparse.ArgumentParser("training for knowledge distillation.")
    p.add_argument("--cfg", type=str, default=[], nargs="*")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--auto-resume", action="store_true",
                   help="resume from <log_path>/latest when it exists")
    p.add_argument("opts", default=None, nargs=argparse.REMAINDER)
    argv = list(sys.argv[1:] if argv is None else argv)
    # `--cfg a.yaml b.yaml KEY VAL`: --cfg takes only *.yaml/*.yml paths, the
    # remaining words are KEY VALUE overrides (argparse's nargs='*' would
    # otherwise swallow them)
    if "--cfg" in argv:
        i = argv.index("--cfg") + 1
        j = i
        while j < len(argv) and argv[j].endswith((".yaml", ".yml")):
            j += 1
        rest = argv[j:]
        flags = [a for a in rest if a in ("--resume", "--auto-resume")]
        rest = [a for a in rest if a not in flags]
        argv = argv[:j] + flags + (["--"] + rest if rest else [])
    ns = p.parse_args(argv)
    if ns.opts and ns.opts[0] == "--":
        ns.opts = ns.opts[1:]
    return ns


def run(argv=None):
    import torch
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.ops.backend import set_backend
    from mdistiller_ddp_amd.parallel import dist as D

    args = parse(argv)
    cfg = get_cfg()
    for f in args.cfg:
        cfg.merge_from_file(f)
    cfg.merge_from_list(args.opts or [])
    info = D.init_distributed(cfg.DIST.BACKEND, float(cfg.DIST.TIMEOUT_S))
    ws = info.world_size
    cfg.EXPERIMENT.DDP = ws > 1
    cfg.DATASET.TEST.BATCH_SIZE = max(1, cfg.DATASET.TEST.BATCH_SIZE // ws)
    cfg.SOLVER.BATCH_SIZE = max(1, cfg.SOLVER.BATCH_SIZE // ws)
    cfg.freeze()
    set_backend(cfg.RUNTIME.BACKEND)
    if cfg.EXPERIMENT.SEED >= 0:
        torch.manual_seed(cfg.EXPERIMENT.SEED)
    if cfg.EXPERIMENT.DETERMINISTIC:
        torch.use_deterministic_algorithms(True, warn_only=True)
    elif info.device.type == "cuda":
        torch.backends.cudnn.benchmark = True
    resume = "auto" if args.auto_resume else args.resume
    try:
        return main(cfg, resume, args.opts, info)
    except KeyboardInterrupt:
        pass
    finally:
        D.destroy()


if __name__ == "__main__":
    run()
