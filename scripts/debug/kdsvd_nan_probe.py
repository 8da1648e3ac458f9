"""Where does KDSVD training go non-finite?  Two graph runs and two eager
runs of the same fp32 steps (same init, same data): per-step loss_kd, grad
norm, finiteness, and the smallest relative eigenvalue gap among the k+3
leading student eigenvalues (the SVD backward divides by it)."""
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
base = build_distiller(cfg, 100, "cuda")
gaps = []
orig_eig = FL._sym_eig


def _eig_spy(g):
    lam, v = orig_eig(g)
    if not torch.cuda.is_current_stream_capturing():
        top = lam[:, :8]
        d = (top[:, :-1] - top[:, 1:]).abs() / top[:, :1].abs().clamp_min(1e-30)
        gaps.append(float(d.min()))
    return lam, v


FL._sym_eig = _eig_spy
finals = []
for run, g in enumerate((True, True, False, False)):
    d = copy.deepcopy(base)
    d.train()
    st = TrainStep(d, cfg, "cuda", use_graph=g, dtype=torch.float32)
    st.set_epoch(1.0)
    ld = SyntheticLoader("cifar100", 16, "cuda", steps_per_epoch=6, channels_last=True)
    for i, b in enumerate(ld):
        gaps.clear()
        preds, losses = st.step(b)
        torch.cuda.synchronize()
        gr = st.flat.grads
        print(f"run {run} graph={g} step {i}: loss_kd {float(losses['loss_kd']):.7g} "
              f"ce {float(losses['loss_ce']):.7g} |g| {float(torch.nan_to_num(gr).norm()):.6g} "
              f"grad finite {bool(torch.isfinite(gr).all())} params finite "
              f"{bool(torch.isfinite(st.flat.data).all())} |p| {float(st.flat.data.double().norm()):.6g} "
              f"min rel gap {min(gaps) if gaps else float('nan'):.3g}", flush=True)
    finals.append(st.flat.data.clone())
for i in range(1, 4):
    rel = (finals[i].double() - finals[0].double()).norm() / finals[0].double().norm()
    print(f"final params run {i} vs run 0: rel {float(rel):.3g}", flush=True)
