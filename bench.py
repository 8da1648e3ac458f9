#!/usr/bin/env python
"""Headline benchmark: DKD ResNet32x4 -> ResNet8x4 on CIFAR-100-shape data.

Metric (BASELINE.json): training images/sec for the whole node at 1/2/4/8
MI355X.  The reference publishes 11 ms/iter at batch 64 on one GPU
(``.github/dkd.png``) = 5,818 img/s; that is ``vs_baseline``'s denominator.

What one timed step contains (nothing skipped): the batch copy into the
step's input buffers, teacher forward (no-grad, BN-folded, own stream),
student forward, fused CE+DKD loss, student backward, gradient all-reduce
over RCCL (N > 1), fused SGD(momentum 0.9, wd 5e-4) update, BN running-stat
updates and on-device metric accumulation -- the full ``TrainStep`` of
the framework's trainer.  Config: configs/cifar100/dkd/res32x4_res8x4.yaml,
per-GPU batch 64 (the config's batch; weak scaling: global = 64 x N),
bf16 compute with fp32 master weights, synthetic device-resident data and
random-init weights (no network for datasets or checkpoints).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 under torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_IMG_S = 64 / 0.011  # 11 ms/iter at batch 64 (.github/dkd.png) = 5818 img/s
CFG_FILE = os.path.join(HERE, "configs", "cifar100", "dkd", "res32x4_res8x4.yaml")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch")
    ap.add_argument("--cfg", default=CFG_FILE)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-teacher-stream", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("opts", nargs=argparse.REMAINDER)
    args = ap.parse_args()

    import torch
    from mdistiller_ddp_amd.ops.backend import set_backend
    from mdistiller_ddp_amd.parallel import dist as D
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    from mdistiller_ddp_amd.runtime import streams

    set_backend(args.backend)
    streams.set_enabled(not args.no_teacher_stream)
    info = D.init_distributed()
    dev = info.device
    if dev.type == "cuda":
        torch.backends.cudnn.benchmark = True
    cfg = get_cfg()
    cfg.merge_from_file(args.cfg)
    if args.opts:
        cfg.merge_from_list(args.opts)
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.freeze()

    torch.manual_seed(1234 + info.rank)
    distiller = build_distiller(cfg, num_classes=100, device=dev, num_data=50000)
    dtype = torch.bfloat16 if (args.dtype == "bf16" and dev.type == "cuda") else torch.float32
    step = TrainStep(distiller, cfg, dev, trainer=cfg.SOLVER.TRAINER,
                     use_graph=not args.no_graph, dtype=dtype)
    distiller.train()
    step.set_epoch(cfg.DKD.WARMUP + 1.0)  # past DKD warm-up: full loss
    step.set_lr(cfg.SOLVER.LR)
    loader = SyntheticLoader("cifar100", args.batch, dev, steps_per_epoch=10 ** 9, pool=8,
                             seed=info.rank, channels_last=(dev.type == "cuda"))
    it = iter(loader)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step.step(next(it))
    sync()
    D.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step.step(next(it))
    sync()
    D.barrier()
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if D.is_dist():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    # sanity: the run trained (finite loss)
    m = step.meters.summary(reduce=True)
    n = info.world_size
    ms = 1000.0 * dt / args.steps
    value = n * args.batch * args.steps / dt
    if info.rank == 0:
        out = {
            "metric": "images/sec (whole node) DKD ResNet32x4->ResNet8x4 CIFAR-100",
            "value": round(value, 1),
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_IMG_S, 3),
            "dtype": "bf16" if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (CIFAR-100 shape 3x32x32, 100 classes, device-resident), random-init weights",
            "config": {
                "model": "DKD resnet32x4->resnet8x4",
                "global_batch": args.batch * n,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "graph": not args.no_graph,
                "backend": args.backend,
                "cfg": os.path.relpath(args.cfg, HERE),
            },
            "final_loss": round(m["loss"], 4),
        }
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
