#!/usr/bin/env python
"""Headline benchmark: DKD ResNet32x4 -> ResNet8x4 on CIFAR-100-shape data.

Metric (BASELINE.json): training images/sec for the whole node at 1/2/4/8
MI355X.  The reference publishes 11 ms/iter at batch 64 on one GPU
(``.github/dkd.png``) = 5,818 img/s; that is ``vs_baseline``'s denominator.

What one timed step contains (nothing skipped): the batch copy into the
step's input buffers, teacher forward (no-grad, BN-folded, own stream),
student forward, fused CE+DKD loss, student backward, gradient all-reduce
over RCCL (N > 1), fused SGD(momentum 0.9, wd 5e-4) update, BN running-stat
updates and on-device metric accumulation -- the framework's TrainStep
(mdistiller_ddp_amd/benchmark.py).  Config:
configs/cifar100/dkd/res32x4_res8x4.yaml, per-GPU batch 64 (the config's
batch; weak scaling: global = 64 x N), bf16 compute with fp32 master
weights, synthetic device-resident data and random-init weights (no network
for datasets or checkpoints).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N > 1 under torch.distributed.run, one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

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
    ap.add_argument("--no-train-kernels", action="store_true",
                    help="student conv+BN through MIOpen instead of the native kernels (A/B)")
    ap.add_argument("opts", nargs=argparse.REMAINDER)
    args = ap.parse_args()

    from mdistiller_ddp_amd import benchmark
    from mdistiller_ddp_amd.ops import nn as mda_nn
    from mdistiller_ddp_amd.parallel import dist as D

    mda_nn.set_train_kernels(not args.no_train_kernels)
    r = benchmark.run(args.cfg, args.batch, args.steps, args.warmup, opts=args.opts,
                      use_graph=not args.no_graph, backend=args.backend, dtype=args.dtype,
                      teacher_stream=not args.no_teacher_stream)
    if r["rank"] == 0:
        n = r["n_gpus"]
        out = {
            "metric": "images/sec (whole node) DKD ResNet32x4->ResNet8x4 CIFAR-100",
            "value": round(r["images_per_s"], 1),
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(r["images_per_s"] / BASELINE_IMG_S, 3),
            "dtype": r["dtype"],
            "data": "synthetic (CIFAR-100 shape 3x32x32, 100 classes, device-resident), random-init weights",
            "config": {
                "model": "DKD resnet32x4->resnet8x4",
                "global_batch": r["global_batch"],
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "graph": r["graph"],
                "backend": args.backend,
                "train_kernels": not args.no_train_kernels,
                "cfg": os.path.relpath(args.cfg, HERE),
            },
            "final_loss": round(r["final_loss"], 4),
        }
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
