#!/usr/bin/env python
"""Intermittent NaN hunt for OFD's graph steps (tests/test_gpu_e2e.py
test_distiller_graph_steps[OFD]): run the same 8-step captured job several
times per arm and count runs whose loss_kd is not finite."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.config import get_cfg  # noqa: E402
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader  # noqa: E402
from mdistiller_ddp_amd.engine.build import build_distiller  # noqa: E402
from mdistiller_ddp_amd.engine.step import TrainStep  # noqa: E402


def run(opts, trials):
    bad = 0
    for t in range(trials):
        torch.manual_seed(t)
        cfg = get_cfg()
        cfg.DISTILLER.TYPE = "OFD"
        cfg.DISTILLER.TEACHER = "resnet32x4"
        cfg.DISTILLER.STUDENT = "resnet8x4"
        cfg.DISTILLER.RANDOM_TEACHER = True
        cfg.merge_from_list(opts)
        d = build_distiller(cfg, 100, "cuda", num_data=2000)
        d.train()
        st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
        st.set_epoch(1.0)
        ld = SyntheticLoader("cifar100", 32, "cuda", steps_per_epoch=8, num_data=2000, channels_last=True)
        per = []
        if os.environ.get("NEXT") == "1":  # hand each step the next batch (look-ahead prefetch)
            bl = list(ld)
            for i, b in enumerate(bl):
                _, losses = st.step(b, next_batch=bl[i + 1] if i + 1 < len(bl) else None)
                per.append(float(losses["loss_kd"]))
        else:
            for b in ld:
                _, losses = st.step(b)
                per.append(float(losses["loss_kd"]))
        torch.cuda.synchronize()
        if not all(v == v for v in per):
            bad += 1
        print("  run", t, ["%.5g" % v for v in per], flush=True)
        del st, d
    return bad


if __name__ == "__main__":
    trials = int(os.environ.get("TRIALS", "4"))
    arms = {
        "default": [],
        "lookahead off": ["RUNTIME.TEACHER_LOOKAHEAD", "off"],
        "teacher eval BN": ["OFD.TEACHER_TRAIN_BN", "False"],
    }
    only = os.environ.get("ARM")
    if only:
        arms = {only: arms[only]}
    for name, opts in arms.items():
        print(f"{name}: {run(opts, trials)} / {trials} runs with NaN loss_kd", flush=True)
