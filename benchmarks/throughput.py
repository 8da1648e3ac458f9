#!/usr/bin/env python
"""Throughput of every BASELINE.json configuration (one JSON row per config).

    python benchmarks/throughput.py [--configs all|dkd_cifar,...] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N benchmarks/throughput.py ...

Rows: config name, images/s for the whole job, ms/step, per-GPU batch,
world size.  All synthetic data of the dataset's shape, random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")  # see mdistiller_ddp_amd/__init__.py
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (yaml, per-GPU batch, extra opts, dataset)
    "kd_cifar_res56_res20": ("configs/cifar100/kd.yaml", 64,
                             ["DISTILLER.TEACHER", "resnet56", "DISTILLER.STUDENT", "resnet20"], None),
    "dkd_cifar_res32x4_res8x4": ("configs/cifar100/dkd/res32x4_res8x4.yaml", 64, [], None),
    "dot_cifar_res32x4_res8x4": ("configs/cifar100/dot/res32x4_res8x4.yaml", 64, [], None),
    "kd_cifar_res32x4_res8x4": ("configs/cifar100/kd.yaml", 64, [], None),
    "crd_cifar_res32x4_res8x4": ("configs/cifar100/crd.yaml", 64, [], None),
    "reviewkd_cifar_res32x4_res8x4": ("configs/cifar100/reviewkd.yaml", 64, [], None),
    "fitnet_cifar_res32x4_res8x4": ("configs/cifar100/fitnet.yaml", 64, [], None),
    "ofd_cifar_res32x4_res8x4": ("configs/cifar100/ofd.yaml", 64, [], None),
    "rkd_cifar_res32x4_res8x4": ("configs/cifar100/rkd.yaml", 64, [], None),
    "at_cifar_res32x4_res8x4": ("configs/cifar100/at.yaml", 64, [], None),
    "nst_cifar_res32x4_res8x4": ("configs/cifar100/nst.yaml", 64, [], None),
    "pkt_cifar_res32x4_res8x4": ("configs/cifar100/pkt.yaml", 64, [], None),
    "sp_cifar_res32x4_res8x4": ("configs/cifar100/sp.yaml", 64, [], None),
    "vid_cifar_res32x4_res8x4": ("configs/cifar100/vid.yaml", 64, [], None),
    "kdsvd_cifar_res32x4_res8x4": ("configs/cifar100/kdsvd.yaml", 64, [], None),
    "vanilla_cifar_res8x4": ("configs/cifar100/vanilla.yaml", 64,
                             ["DISTILLER.STUDENT", "resnet8x4"], None),
    "dkd_cifar_vgg13_vgg8": ("configs/cifar100/dkd/vgg13_vgg8.yaml", 64, [], None),
    "dkd_cifar_wrn40_2_wrn16_2": ("configs/cifar100/dkd/wrn40_2_wrn_16_2.yaml", 64, [], None),
    "dkd_cifar_res32x4_shuv1": ("configs/cifar100/dkd/res32x4_shuv1.yaml", 64, [], None),
    "dkd_cifar_vgg13_mv2": ("configs/cifar100/dkd/vgg13_mv2.yaml", 64, [], None),
    "reviewkd_imagenet_r34_r18": ("configs/imagenet/r34_r18/reviewkd.yaml", 32, [], None),
    "dkd_imagenet_r50_mv1": ("configs/imagenet/r50_mv1/dkd.yaml", 64, [], None),
    # the DOT configurations of the reference README (BASELINE.md accuracy table)
    "dot_cifar_vgg13_vgg8": ("configs/cifar100/dot/vgg13_vgg8.yaml", 64, [], None),
    "dot_cifar_res32x4_shuv2": ("configs/cifar100/dot/res32x4_shuv2.yaml", 64, [], None),
    "dot_tiny_r18_mv2": ("configs/tiny_imagenet/dot/r18_mv2.yaml", 256, [], None),
    "dot_tiny_r18_shuv2": ("configs/tiny_imagenet/dot/r18_shuv2.yaml", 256, [], None),
}


# reference "training time (ms)" per iteration at batch 64, `.github/dkd.png`
# inset, CIFAR-100 ResNet32x4 -> ResNet8x4, unstated GPU
BASELINE_MS = {"kd_cifar_res32x4_res8x4": 11.0, "dkd_cifar_res32x4_res8x4": 11.0,
               "fitnet_cifar_res32x4_res8x4": 14.0, "ofd_cifar_res32x4_res8x4": 19.0,
               "rkd_cifar_res32x4_res8x4": 25.0, "reviewkd_cifar_res32x4_res8x4": 26.0,
               "crd_cifar_res32x4_res8x4": 41.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="all")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--out", default=None, help="append JSON rows to this file")
    ap.add_argument("--opts", nargs="*", default=[], help="extra KEY VALUE config overrides for every row")
    ap.add_argument("--in-process", action="store_true",
                    help="run every config in THIS process (default: one child process each)")
    args = ap.parse_args()
    names = list(CONFIGS) if args.configs == "all" else args.configs.split(",")
    if len(names) > 1 and not args.in_process and "WORLD_SIZE" not in os.environ:
        # one fresh process per config: a step's streams get hardware queues by
        # the process's history of stream creation, and a config measured after
        # others in the same process can run up to 40 % slower
        # (profiles/r3_dot_history.md) -- rows then depend on the run order
        import subprocess
        for name in names:
            cmd = [sys.executable, os.path.abspath(__file__), "--configs", name, "--steps",
                   str(args.steps), "--warmup", str(args.warmup), "--in-process"]
            if args.no_graph:
                cmd.append("--no-graph")
            if args.out:
                cmd += ["--out", args.out]
            if args.opts:
                cmd += ["--opts"] + list(args.opts)
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
            rows = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(rows[-1] if rows else json.dumps({"config": name, "error": f"exit {r.returncode}"}),
                  flush=True)
        return
    from mdistiller_ddp_amd import benchmark
    for name in names:
        yaml, bs, opts, ds = CONFIGS[name]
        try:
            r = benchmark.run(os.path.join(ROOT, yaml), bs, args.steps, args.warmup,
                              opts=list(opts) + list(args.opts),
                              use_graph=not args.no_graph, dataset=ds)
        except Exception as e:  # report and continue with the other configs
            print(json.dumps({"config": name, "error": f"{type(e).__name__}: {e}"[:300]}), flush=True)
            continue
        if r["rank"] == 0:
            row = {"config": name, "images_per_s": round(r["images_per_s"], 1),
                   "ms_per_step": round(r["ms_per_step"], 3), "per_gpu_batch": bs,
                   "n_gpus": r["n_gpus"], "graph": r["graph"], "dtype": r["dtype"],
                   "final_loss": round(r["final_loss"], 4),
                   "host_ms_per_step": round(r["host_ms_per_step"], 3),
                   "host_idle_ms_per_step": round(r["host_idle_ms_per_step"], 3)}
            if name in BASELINE_MS and r["n_gpus"] == 1 and bs == 64:
                row["baseline_ms"] = BASELINE_MS[name]
                row["speedup_vs_baseline"] = round(BASELINE_MS[name] / r["ms_per_step"], 2)
            print(json.dumps(row), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
