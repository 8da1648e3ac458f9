"""Engine on CPU (world_size 1): milestone A (KD resnet56 -> resnet20 on
CIFAR-shape synthetic data), checkpoint format, resume equivalence, LR
schedules, DOT / CRD trainers."""
import os

import pytest
import torch

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.data import get_dataset
from mdistiller_ddp_amd.engine import trainer_dict, build_distiller, adjust_learning_rate
from mdistiller_ddp_amd.engine.utils import load_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp_path, yaml="configs/cifar100/kd.yaml", **over):
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, yaml))
    cfg.DISTILLER.TEACHER = over.pop("teacher", "resnet56")
    cfg.DISTILLER.STUDENT = over.pop("student", "resnet20")
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.DATASET.SYNTHETIC = True
    cfg.DATASET.SYNTHETIC_SIZE = 96
    cfg.DATASET.TEST.BATCH_SIZE = 32
    cfg.SOLVER.BATCH_SIZE = 32
    cfg.SOLVER.EPOCHS = over.pop("epochs", 2)
    cfg.LOG.PREFIX = str(tmp_path)
    cfg.EXPERIMENT.SEED = 0
    cfg.CRD.NCE.K = 64
    for k, v in over.items():
        cfg.merge_from_list([k, v])
    return cfg


def _run(cfg, name="exp", resume=False):
    torch.manual_seed(0)
    tr, va, n, nc = get_dataset(cfg, torch.device("cpu"))
    d = build_distiller(cfg, nc, "cpu", n)
    t = trainer_dict[cfg.SOLVER.TRAINER](name, d, tr, va, cfg, device=torch.device("cpu"))
    t.train(resume=resume)
    return t


def test_milestone_a_kd_res56_res20(tmp_path):
    cfg = _cfg(tmp_path)
    cfg.freeze()
    t = _run(cfg)
    out = tmp_path / "exp"
    for f in ("latest", "student_latest", "best", "student_best", "worklog.txt", "worklog.yaml",
              "code/_cfg.yaml", "code/distiller.py"):
        assert (out / f).exists(), f
    st = load_checkpoint(str(out / "latest"))
    assert st["epoch"] == 2 and set(st) == {"epoch", "model", "optimizer", "best_acc"}
    assert all(k.startswith("module.") for k in st["model"])
    assert any(k.startswith("module.teacher.") for k in st["model"])
    assert "momentum_buffer" in st["optimizer"]["state"][0]
    stu = load_checkpoint(str(out / "student_latest"))
    assert set(stu) == {"model"} and "fc.weight" in stu["model"]
    txt = (out / "worklog.txt").read_text()
    assert "best_acc" in txt and "test_acc_top5" in txt


def test_resume_equivalence(tmp_path):
    """2 epochs straight == 1 epoch + --resume + 1 epoch (bitwise on CPU)."""
    cfg = _cfg(tmp_path / "a", epochs=2)
    cfg.freeze()
    straight = _run(cfg)
    cfg1 = _cfg(tmp_path / "b", epochs=1)
    cfg1.freeze()
    _run(cfg1)
    cfg2 = _cfg(tmp_path / "b", epochs=2)
    cfg2.freeze()
    resumed = _run(cfg2, resume=True)
    a = straight.distiller.student.state_dict()
    b = resumed.distiller.student.state_dict()
    for k in a:
        torch.testing.assert_close(b[k], a[k], rtol=0, atol=0, msg=k)


@pytest.mark.parametrize("yaml,trainer,typ", [
    ("configs/cifar100/dot/res32x4_res8x4.yaml", "dot", "KD"),
    ("configs/cifar100/crd.yaml", "crd", "CRD"),
    ("configs/cifar100/dkd/res32x4_res8x4.yaml", "base", "DKD"),
    ("configs/cifar100/reviewkd.yaml", "base", "REVIEWKD"),
    ("configs/cifar100/vanilla.yaml", "base", "NONE"),
])
def test_trainers_run(tmp_path, yaml, trainer, typ):
    cfg = _cfg(tmp_path, yaml, teacher="resnet32x4", student="resnet8x4", epochs=1)
    assert cfg.SOLVER.TRAINER == trainer and cfg.DISTILLER.TYPE == typ
    cfg.freeze()
    t = _run(cfg)
    assert (tmp_path / "exp" / "latest").exists()
    assert t.best_acc >= 0


def test_crd_dot_trainer(tmp_path):
    cfg = _cfg(tmp_path, "configs/cifar100/crd.yaml", teacher="resnet32x4", student="resnet8x4",
               epochs=1)
    cfg.SOLVER.TRAINER = "crd_dot"
    cfg.freeze()
    _run(cfg)


def test_lr_schedules():
    cfg = get_cfg()
    cfg.SOLVER.LR = 0.05
    cfg.SOLVER.SCHEDULE.MULTISTEP.STAGES = [150, 180, 210]
    assert adjust_learning_rate(150, 0, cfg, 100) == pytest.approx(0.05)
    assert adjust_learning_rate(151, 3, cfg, 100) == pytest.approx(0.005)
    assert adjust_learning_rate(240, 0, cfg, 100) == pytest.approx(0.00005)
    cfg.SOLVER.SCHEDULE.TYPE = "COSINE"
    cfg.SOLVER.EPOCHS = 10
    cfg.SOLVER.SCHEDULE.COSINE.WARMUP = 2
    cfg.SOLVER.SCHEDULE.COSINE.RATE = 0.01
    nb = 50
    assert adjust_learning_rate(1, 0, cfg, nb) == pytest.approx(0.05 / 100)
    assert adjust_learning_rate(2, 49, cfg, nb) == pytest.approx(0.05)
    assert adjust_learning_rate(3, 0, cfg, nb) == pytest.approx(0.05)
    mid = adjust_learning_rate(7, 0, cfg, nb)
    assert mid == pytest.approx(0.5 * (0.05 - 0.0005) + 0.0005)
    assert adjust_learning_rate(10, 49, cfg, nb) > 0.0005


def test_fault_injection_raises(tmp_path):
    cfg = _cfg(tmp_path, epochs=1)
    cfg.RUNTIME.FAULT_INJECT = "0:2"
    cfg.freeze()
    with pytest.raises(RuntimeError, match="injected fault"):
        _run(cfg)


def test_cli_train_and_auto_resume(tmp_path):
    import subprocess
    import sys
    base = ["--cfg", os.path.join(ROOT, "configs/cifar100/kd.yaml"), "DISTILLER.TEACHER", "resnet56",
            "DISTILLER.STUDENT", "resnet20", "DISTILLER.RANDOM_TEACHER", "True",
            "DATASET.SYNTHETIC", "True", "DATASET.SYNTHETIC_SIZE", "64", "SOLVER.BATCH_SIZE", "32",
            "DATASET.TEST.BATCH_SIZE", "32", "LOG.PREFIX", str(tmp_path), "EXPERIMENT.NAME", "cli"]
    env = dict(os.environ, MDA_BACKEND="torch")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/train.py")] + base +
                       ["SOLVER.EPOCHS", "2"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(list(tmp_path.rglob("latest"))) == 1
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/train.py")] + base[:2] +
                       ["--auto-resume"] + base[2:] + ["SOLVER.EPOCHS", "2"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resumed from" in r.stdout and "at epoch 3" in r.stdout


def test_topk_rank_breaks_ties_like_stable_sort():
    import torch
    from mdistiller_ddp_amd.engine.step import topk_rank
    g = torch.Generator().manual_seed(0)
    preds = torch.randint(0, 4, (256, 20), generator=g).float()
    target = torch.randint(0, 20, (256,), generator=g)
    order = torch.argsort(-preds, dim=1, stable=True)
    want = (order == target.reshape(-1, 1)).float().argmax(1)
    assert torch.equal(topk_rank(preds, target), want)


import pytest


@pytest.mark.parametrize("trainer,typ", [("base", "DKD"), ("dot", "KD"), ("base", "REVIEWKD")])
def test_every_learnable_param_is_updated(trainer, typ):
    """Every parameter that a loss reaches moves after a step (the reachability
    walk that skips grad-less params must find all of them)."""
    import torch
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep, autograd_reachable
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = typ
    cfg.DISTILLER.TEACHER = "resnet20"
    cfg.DISTILLER.STUDENT = "resnet8"
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.SOLVER.TRAINER = trainer
    if typ == "REVIEWKD":
        cfg.REVIEWKD.IN_CHANNELS = [16, 32, 64, 64]
        cfg.REVIEWKD.OUT_CHANNELS = [16, 32, 64, 64]
    torch.manual_seed(0)
    d = build_distiller(cfg, 100, "cpu")
    d.train()
    st = TrainStep(d, cfg, "cpu", trainer=trainer)
    st.set_epoch(5.0)
    before = [p.detach().clone() for p in st.flat.params]
    for b in SyntheticLoader("cifar100", 8, "cpu", steps_per_epoch=2):
        st.step(b)
    names = {id(p): n for n, p in d.named_parameters()}
    stuck = [names[id(p)] for p, b0 in zip(st.flat.params, before) if torch.equal(p.detach(), b0)]
    assert not stuck, stuck
