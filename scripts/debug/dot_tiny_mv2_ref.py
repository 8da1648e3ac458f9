"""DOT Tiny-ImageNet MobileNetV2: single-pass and two-pass bf16 gradients of
one step, each against an fp32 PyTorch two-pass reference (NCHW, eager).
If the single pass is as close to fp32 as the two-pass bf16 run is, their
mutual difference is bf16 noise, not a wrong gradient."""
import copy
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
from mdistiller_ddp_amd.ops.backend import use_backend

student = sys.argv[1] if len(sys.argv) > 1 else "MobileNetV2"
data = sys.argv[2] if len(sys.argv) > 2 else "tiny_imagenet"
teacher = sys.argv[3] if len(sys.argv) > 3 else "ResNet18"
ncls = {"tiny_imagenet": 200, "cifar100": 100}[data]


def cfg_(single):
    c = get_cfg()
    c.DATASET.TYPE = data
    c.DISTILLER.TYPE = "KD"
    c.DISTILLER.TEACHER = teacher
    c.DISTILLER.STUDENT = student
    c.DISTILLER.RANDOM_TEACHER = True
    c.SOLVER.TRAINER = "dot"
    c.RUNTIME.DOT_SINGLE_PASS = "true" if single else "false"
    return c


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


torch.manual_seed(0)
d0 = build_distiller(cfg_(True), ncls, "cuda")
batch = next(iter(SyntheticLoader(data, 32, "cuda", steps_per_epoch=1, channels_last=False)))
grads = []
for single, dt, be in ((True, torch.bfloat16, "auto"), (False, torch.bfloat16, "auto")):
    d = copy.deepcopy(d0)
    with use_backend(be):
        d.train()
        cl = be != "torch"
        st = TrainStep(d, cfg_(single), "cuda", trainer="dot", use_graph=False, dtype=dt,
                       channels_last=cl)
        st.set_epoch(1.0)
        b = {k: (v.contiguous(memory_format=torch.channels_last) if (cl and v.dim() == 4) else v.clone())
             for k, v in batch.items()}
        st.step(b)
        torch.cuda.synchronize()
        grads.append(st.flat.grads.clone())
names = {id(p): n for n, p in d.named_parameters()}
for k in (0, 1):
    g1, g2 = grads[0][k], grads[1][k]
    tot = (g1 - g2).norm().item() ** 2
    rows = []
    for p, o in zip(st.flat.params, st.flat.offsets):
        a, b = g1[o:o + p.numel()], g2[o:o + p.numel()]
        rows.append(((a - b).norm().item() ** 2 / max(tot, 1e-30), names.get(id(p), "?"),
                     b.norm().item() / g2.norm().item(), rel(a, b)))
    rows.sort(reverse=True)
    print(f"set {k}: single vs two {rel(g1, g2):.4g}; top error shares:", flush=True)
    for r in rows[:8]:
        print(f"   {r[1]}: share {r[0]:.3f}, norm frac {r[2]:.3g}, rel {r[3]:.3g}", flush=True)
