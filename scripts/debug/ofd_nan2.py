#!/usr/bin/env python
"""Which tensor goes non-finite first in OFD's recaptured step (see ofd_nan.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.config import get_cfg  # noqa: E402
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader  # noqa: E402
from mdistiller_ddp_amd.engine.build import build_distiller  # noqa: E402
from mdistiller_ddp_amd.engine.step import TrainStep  # noqa: E402
from mdistiller_ddp_amd.distillers import OFD as OFDmod  # noqa: E402

torch.manual_seed(0)
cfg = get_cfg()
cfg.DISTILLER.TYPE = "OFD"
cfg.DISTILLER.TEACHER = "resnet32x4"
cfg.DISTILLER.STUDENT = "resnet8x4"
cfg.DISTILLER.RANDOM_TEACHER = True
d = build_distiller(cfg, 100, "cuda", num_data=2000)
d.train()
st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
st.set_epoch(1.0)
orig = d.ofd_loss
step = [0]


def fin(t):
    return bool(torch.isfinite(t.float()).all().item()) if isinstance(t, torch.Tensor) else True


def probe(fs, ft):
    if not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream().synchronize()
        print(f"  step {step[0]}: student preacts finite {[fin(x) for x in fs]} teacher preacts finite "
              f"{[fin(x) for x in ft]} teacher absmax {[float(x.float().abs().max()) for x in ft if isinstance(x, torch.Tensor)]}",
              flush=True)
    return orig(fs, ft)


d.ofd_loss = probe
ld = SyntheticLoader("cifar100", 32, "cuda", steps_per_epoch=8, num_data=2000, channels_last=True)
for b in ld:
    step[0] += 1
    _, losses = st.step(b)
    torch.cuda.synchronize()
    print(f"step {step[0]} loss_kd {float(losses['loss_kd']):.4g} graphs {st._graphs is not None} "
          f"lookahead {st.lookahead}", flush=True)
for n, m in d.teacher.named_modules():
    if isinstance(m, torch.nn.BatchNorm2d) and not torch.isfinite(m.running_var).all():
        print("non-finite teacher running_var:", n)
        break
