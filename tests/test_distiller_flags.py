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
def test_ofd_graph_capturable_follows_teacher_bn_mode(train_bn):
    # train-mode teacher BN stays eager (profiles/r1_ofd_graph_ab.md)
    d = _ofd(train_bn)
    assert d.graph_capturable is (not train_bn)


def test_ofd_train_bn_teacher_runs_fp32_under_autocast():
    d = _ofd(True)
    d.train()
    assert d.teacher.training
    x = torch.randn(2, 3, 32, 32)
    out = d.teacher_forward(x).get()
    logits = out[0]
    assert logits.dtype == torch.float32 and torch.isfinite(logits).all()
