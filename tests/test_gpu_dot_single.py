"""DOT in one backward pass (engine/step.py ``_dot_single_backward``,
ops/hip_train.py ``_Dual``): the KD and task cotangents stacked along the batch
through every native backward kernel must give the same two gradient sets as
the reference's two backward passes (reference engine/trainer.py:425-432)."""
import copy

import pytest
import torch

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader

pytestmark = pytest.mark.gpu


def _cfg(student, single, teacher="resnet32x4", data="cifar100"):
    cfg = get_cfg()
    cfg.DATASET.TYPE = data
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = teacher
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.SOLVER.TRAINER = "dot"
    cfg.RUNTIME.DOT_SINGLE_PASS = "true" if single else "false"
    return cfg


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


# vgg8: biased convs (zero gradient in front of a training BN), native max pools,
# ReLU inside the conv launch (models/cifar/vgg.py); ResNet18: the ImageNet stem's
# 7x7 conv and 3x3 / stride-2 max pool (configs/imagenet/r34_r18/dot.yaml);
# MobileNetV2 (CIFAR and Tiny-ImageNet): depthwise convs, residual forks, the
# fused head (a 1x1-conv classifier on Tiny-ImageNet)
_STUDENTS = {"resnet8x4": ("resnet32x4", "cifar100", 100, 64),
             "resnet20": ("resnet32x4", "cifar100", 100, 64),
             "resnet32x4": ("resnet32x4", "cifar100", 100, 64),
             "vgg8": ("vgg13", "cifar100", 100, 64),
             "MobileNetV2": ("vgg13", "cifar100", 100, 64),
             "MobileNetV2_tiny": ("ResNet18", "tiny_imagenet", 200, 32),
             "ResNet18": ("ResNet34", "imagenet", 1000, 16)}


@pytest.mark.parametrize("student", list(_STUDENTS))
def test_single_pass_gradients_match_two_passes(student):
    teacher, data, ncls, bs = _STUDENTS[student]
    student_id, student = student, student.replace("_tiny", "")
    torch.manual_seed(0)
    d1 = build_distiller(_cfg(student, True, teacher, data), ncls, "cuda")
    d2 = copy.deepcopy(d1)
    ld = SyntheticLoader(data, bs, "cuda", steps_per_epoch=1, channels_last=True)
    batch = next(iter(ld))
    grads = []
    for d, single in ((d1, True), (d2, False)):
        d.train()
        st = TrainStep(d, _cfg(student, single, teacher, data), "cuda", trainer="dot", use_graph=False,
                       dtype=torch.bfloat16)
        assert st.dot_single == single
        st.set_epoch(1.0)
        st.step({k: v.clone() for k, v in batch.items()})
        torch.cuda.synchronize()
        grads.append(st.flat.grads.clone())
    names = {id(p): n for n, p in d.named_parameters()}  # (d, st: the last run's)
    flat = st.flat
    for k in (0, 1):  # per-parameter report of the worst layers (diagnostics)
        worst = sorted(((_rel(grads[0][k][o:o + p.numel()], grads[1][k][o:o + p.numel()]),
                         names.get(id(p), "?")) for p, o in zip(flat.params, flat.offsets)
                        if grads[1][k][o:o + p.numel()].abs().sum() > 0), reverse=True)[:8]
        print(f"{student} set {k} worst: " + ", ".join(f"{n} {r:.3g}" for r, n in worst))
    for k in (0, 1):  # row 0: task (CE) gradients, row 1: KD gradients
        assert grads[0][k].abs().sum() > 0
        print(f"{student} set {k}: single/two-pass gradient rel {_rel(grads[0][k], grads[1][k]):.3g}")
        # Tiny-ImageNet MobileNetV2 (17 blocks, 64x64 maps, ReLU6): the 2N-image
        # launches take other tile / split plans than the N-image ones and the
        # bf16 rounding differences grow along the backward -- 1.5-2 % per layer
        # at the input end, ~0 at the head end, spread over every layer
        # (scripts/debug/dot_tiny_mv2_ref.py), not one wrong layer
        tol = 3e-2 if student_id == "MobileNetV2_tiny" else 1e-2
        assert _rel(grads[0][k], grads[1][k]) < tol, (k, _rel(grads[0][k], grads[1][k]))


def test_single_pass_graph_tracks_two_pass_eager():
    """20 steps.  The single-pass hipGraph replay == the single-pass eager
    steps, and the single-pass trajectory is as close to an fp32 PyTorch
    two-pass reference (NCHW, eager) as the bf16 two-pass one is: the two bf16
    runs round differently (the dgrad over 2N images may take another tile /
    split plan), and bf16 noise grows over the steps."""
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(0)
    d0 = build_distiller(_cfg("resnet8x4", True), 100, "cuda")
    ds = [copy.deepcopy(d0) for _ in range(4)]
    outs = []
    runs = ((False, False, torch.bfloat16, "auto"), (True, False, torch.bfloat16, "auto"),
            (True, True, torch.bfloat16, "auto"), (False, False, torch.float32, "torch"))
    for d, (single, g, dt, be) in zip(ds, runs):
        with use_backend(be):
            d.train()
            cl = be != "torch"
            st = TrainStep(d, _cfg("resnet8x4", single), "cuda", trainer="dot", use_graph=g,
                           dtype=dt, channels_last=cl)
            assert st.dot_single == (single and dt == torch.bfloat16)
            st.set_epoch(30.0)
            ld = SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=20, channels_last=cl)
            for b in ld:
                st.step(b)
            torch.cuda.synchronize()
            assert (st._graphs is not None) == g and st._dual is None
            outs.append(st.flat.data.clone())
    two, one, one_g, ref = outs
    r_graph = _rel(one_g, one)
    r_two, r_one = _rel(two, ref), _rel(one, ref)
    print(f"single graph/eager {r_graph:.3g}; vs fp32: two-pass {r_two:.3g} single {r_one:.3g}")
    assert r_graph < 1e-3, r_graph
    assert r_one <= 1.5 * r_two + 2e-3, (r_one, r_two)
