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
configs/cifar100/dkd/res32x4_res8x4.yaml, bf16 compute with fp32 master
weights, synthetic device-resident data and random-init weights (no network
for datasets or checkpoints).

Scaling modes:
  weak   (default) per-GPU batch fixed (``--batch``, default 64 = the config's
         batch); global batch = 64 x N.
  strong global batch fixed (``--global-batch``, default 64 = the reference's
         DDP semantics, tools/train.py:124 divides it by world size); per-GPU
         batch = 64 / N.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
  N > 1 either under torch.distributed.run (one rank per GPU; WORLD_SIZE must
  equal N) or stand-alone, in which case this script launches the N ranks
  itself (a child ``torch.distributed.run``) before touching any GPU and
  exits with its status.
"""
from __future__ import annotations

import argparse
import json
import os

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see mdistiller_ddp_amd/__init__.py
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_IMG_S = 64 / 0.011  # 11 ms/iter at batch 64 (.github/dkd.png) = 5818 img/s
CFG_FILE = os.path.join(HERE, "configs", "cifar100", "dkd", "res32x4_res8x4.yaml")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(n: int) -> int:
    """Run this script under torch.distributed.run with ``n`` ranks (child process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--batch", type=int, default=64, help="per-GPU batch (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=64, help="global batch (strong scaling)")
    ap.add_argument("--cfg", default=CFG_FILE)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-teacher-stream", action="store_true")
    ap.add_argument("--no-train-kernels", action="store_true",
                    help="student conv+BN through MIOpen instead of the native kernels (A/B)")
    ap.add_argument("opts", nargs=argparse.REMAINDER)
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        # stand-alone multi-GPU request: launch the ranks BEFORE any GPU call
        sys.exit(_self_launch(args.gpus))
    world = int(world_env or 1)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; refusing to "
                         f"report a {world}-rank run as {args.gpus} GPUs")
    if args.scaling == "strong":
        if args.global_batch % world:
            raise SystemExit(f"--global-batch {args.global_batch} not divisible by {world} ranks")
        per_gpu = args.global_batch // world
    else:
        per_gpu = args.batch

    import torch
    if world > 1 and torch.cuda.device_count() and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks but only {torch.cuda.device_count()} GPUs visible")

    from mdistiller_ddp_amd import benchmark
    from mdistiller_ddp_amd.ops import nn as mda_nn
    from mdistiller_ddp_amd.parallel import dist as D

    mda_nn.set_train_kernels(not args.no_train_kernels)
    r = benchmark.run(args.cfg, per_gpu, args.steps, args.warmup, opts=args.opts,
                      use_graph=not args.no_graph, backend=args.backend, dtype=args.dtype,
                      teacher_stream=not args.no_teacher_stream, check_replicas=True)
    if r["rank"] == 0:
        n = r["n_gpus"]
        if n != args.gpus:
            raise SystemExit(f"bench.py: measured on {n} ranks, asked for {args.gpus}")
        # the BASELINE metric / model names only for the flagship config; any
        # other --cfg is labelled by its file and has no baseline ratio
        flagship = os.path.realpath(args.cfg) == os.path.realpath(CFG_FILE)
        cfg_name = os.path.relpath(args.cfg, HERE)
        out = {
            "metric": ("images/sec (whole node) DKD ResNet32x4->ResNet8x4 CIFAR-100" if flagship
                       else f"images/sec (whole node) {cfg_name}"),
            "value": round(r["images_per_s"], 1),
            "unit": "images/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": round(r["images_per_s"] / BASELINE_IMG_S, 3) if flagship else None,
            "dtype": r["dtype"],
            "data": "synthetic (CIFAR-100 shape 3x32x32, 100 classes, device-resident), random-init weights (random teacher classifier rescaled to logit std 4)",
            "config": {
                "model": "DKD resnet32x4->resnet8x4" if flagship else cfg_name,
                "global_batch": r["global_batch"],
                "per_gpu_batch": per_gpu,
                "seq_len": None,
                "parallelism": f"dp{n}",
                "graph": r["graph"],
                "graph_comm": r.get("graph_comm"),
                "backend": args.backend,
                "comm_backend": r.get("comm_backend"),
                "train_kernels": not args.no_train_kernels,
                "cfg": os.path.relpath(args.cfg, HERE),
            },
            "replicas_identical": r.get("replicas_identical"),
            "final_loss": round(r["final_loss"], 4),
            "host_ms_per_step": round(r["host_ms_per_step"], 4),
            "host_idle_ms_per_step": round(r["host_idle_ms_per_step"], 4),
        }
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    main()
