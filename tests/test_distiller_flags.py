"""Per-distiller step flags that TrainStep reads (CPU)."""
import os

import pytest
import torch

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.engine.build import build_distiller

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ofd(train_bn):
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs/cifar100/ofd.yaml"))
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.OFD.TEACHER_TRAIN_BN = train_bn
    return build_distiller(cfg, 100, torch.device("cpu"))


@pytest.mark.parametrize("train_bn", [True, False])
def test_ofd_step_is_capturable_in_both_teacher_bn_modes(train_bn):
    # the train-mode teacher BN runs on capture-safe native kernels on the GPU
    d = _ofd(train_bn)
    assert d.graph_capturable


@pytest.mark.parametrize("train_bn", [True, False])
def test_ofd_teacher_bn_mode_and_running_stats(train_bn):
    d = _ofd(train_bn)
    d.train()
    assert d.teacher.training is train_bn
    rm = d.teacher.bn1.running_mean.clone()
    out = d.teacher_forward(torch.randn(2, 3, 32, 32)).get()
    assert torch.isfinite(out[0]).all()
    # reference OFD.train() leaves the teacher BN in train mode: running stats move
    assert (not torch.equal(rm, d.teacher.bn1.running_mean)) is train_bn
