"""Where does KDSVD training go non-finite with the fused post-processing?
Eager fp32 steps, fused vs PyTorch composition, loss + grad norms per step."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mdistiller_ddp_amd.config import get_cfg  # noqa: E402
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader  # noqa: E402
from mdistiller_ddp_amd.engine.build import build_distiller  # noqa: E402
from mdistiller_ddp_amd.engine.step import TrainStep  # noqa: E402
from mdistiller_ddp_amd.ops import feat_losses as FL  # noqa: E402

torch.manual_seed(0)
cfg = get_cfg()
cfg.DISTILLER.TYPE = "KDSVD"
cfg.DISTILLER.TEACHER = "resnet32x4"
cfg.DISTILLER.STUDENT = "resnet8x4"
cfg.DISTILLER.RANDOM_TEACHER = True
d1 = build_distiller(cfg, 100, "cuda")
d2 = copy.deepcopy(d1)
orig = FL.kdsvd_loss
d3 = copy.deepcopy(d1)
for d, fused, g in ((d1, True, True), (d2, False, True), (d3, True, False)):
    FL.kdsvd_loss = (lambda *a, _f=fused, **k: orig(*a, fused=_f, **k))
    d.train()
    st = TrainStep(d, cfg, "cuda", use_graph=g, dtype=torch.float32)
    st.set_epoch(1.0)
    ld = SyntheticLoader("cifar100", 16, "cuda", steps_per_epoch=6, channels_last=True)
    for i, b in enumerate(ld):
        preds, losses = st.step(b)
        torch.cuda.synchronize()
        g = st.flat.grads
        print(f"fused={fused} graph={g} step {i}: loss_kd {float(losses['loss_kd']):.5g} ce {float(losses['loss_ce']):.4g} "
              f"grad finite {bool(torch.isfinite(g).all())} |g| {float(torch.nan_to_num(g).norm()):.4g} "
              f"params finite {bool(torch.isfinite(st.flat.data).all())}", flush=True)
FL.kdsvd_loss = orig
