#!/usr/bin/env python
"""Intermittent non-finite parameters in test_graph_matches_eager[base]
(KD r32x4 -> r8x4, graph replay): run the captured step several times and
report the first step whose parameters or loss are non-finite, plus the
BN grid-barrier error word."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.config import get_cfg  # noqa: E402
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader  # noqa: E402
from mdistiller_ddp_amd.engine.build import build_distiller  # noqa: E402
from mdistiller_ddp_amd.engine.step import TrainStep  # noqa: E402
from mdistiller_ddp_amd.ops import hip_train  # noqa: E402

bad = 0
trials = int(os.environ.get("TRIALS", "3"))
for t in range(trials):
    torch.manual_seed(t)
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = "resnet8x4"
    cfg.DISTILLER.RANDOM_TEACHER = True
    d = build_distiller(cfg, 100, "cuda")
    d.train()
    st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
    st.set_epoch(1.0)
    first = None
    for i, b in enumerate(SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=12, channels_last=True)):
        st.step(b)
        torch.cuda.synchronize()
        if first is None and not torch.isfinite(st.flat.data).all():
            first = i
    errs = hip_train.slot_errors()
    print(f"trial {t}: first non-finite step {first}, barrier errors {errs}, "
          f"fwd finishes {hip_train.bn_finish_count()}, bwd finishes {hip_train.bn_bwd_finish_count()}",
          flush=True)
    bad += first is not None
print(f"{bad} / {trials} trials non-finite")
