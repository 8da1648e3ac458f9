"""Config system: yacs-compatible merge semantics over every shipped YAML."""
import glob
import os

import pytest

from mdistiller_ddp_amd.config import get_cfg, load_cfg, dump_cfg, METHOD_NODES
from mdistiller_ddp_amd.distillers import distiller_dict
from mdistiller_ddp_amd.engine import trainer_dict
from mdistiller_ddp_amd.models import cifar_model_dict, tiny_imagenet_model_dict, imagenet_model_dict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
YAMLS = sorted(glob.glob(os.path.join(ROOT, "configs", "**", "*.yaml"), recursive=True))


def test_all_reference_configs_present():
    assert len(YAMLS) == 45


@pytest.mark.parametrize("path", YAMLS, ids=lambda p: os.path.relpath(p, ROOT))
def test_yaml_merges_and_resolves(path):
    cfg = get_cfg()
    cfg.merge_from_file(path)
    cfg.freeze()
    if "optim" in path:
        return  # overlay files
    assert cfg.DISTILLER.TYPE in distiller_dict
    assert cfg.SOLVER.TRAINER in trainer_dict
    table = {"cifar100": cifar_model_dict, "tiny_imagenet": tiny_imagenet_model_dict,
             "imagenet": imagenet_model_dict}[cfg.DATASET.TYPE]
    assert cfg.DISTILLER.STUDENT in table
    if cfg.DISTILLER.TYPE != "NONE":
        assert cfg.DISTILLER.TEACHER in table


def test_overlay_two_cfgs():
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs/imagenet/r34_r18/kd.yaml"))
    cfg.merge_from_file(os.path.join(ROOT, "configs/imagenet/optim/adamw.yaml"))
    assert cfg.SOLVER.TYPE == "AdamW" and cfg.SOLVER.SCHEDULE.TYPE == "COSINE"


def test_unknown_key_rejected():
    cfg = get_cfg()
    with pytest.raises(KeyError):
        cfg.merge_from_other_cfg(load_cfg("SOLVER:\n  NOT_A_KEY: 1\n"))
    with pytest.raises(KeyError):
        cfg.merge_from_list(["DKD.GAMMA", "1.0"])


def test_opts_override_and_coercion():
    cfg = get_cfg()
    cfg.merge_from_list(["SOLVER.LR", "0.1", "DKD.WARMUP", "5", "SOLVER.SCHEDULE.MULTISTEP.STAGES",
                         "[1, 2]", "DKD.BETA", "2"])
    assert cfg.SOLVER.LR == 0.1 and cfg.DKD.WARMUP == 5
    assert cfg.SOLVER.SCHEDULE.MULTISTEP.STAGES == [1, 2]
    assert isinstance(cfg.DKD.BETA, float) and cfg.DKD.BETA == 2.0
    with pytest.raises(ValueError):
        cfg.merge_from_list(["SOLVER.LR", "'abc'"])


def test_freeze_and_dump_roundtrip():
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs/cifar100/dkd/res32x4_res8x4.yaml"))
    cfg.freeze()
    with pytest.raises(AttributeError):
        cfg.SOLVER.LR = 1.0
    d = dump_cfg(cfg)
    assert "DKD" in d and "KD" not in d and "CRD" not in d
    again = get_cfg()
    again.merge_from_other_cfg(load_cfg(cfg.dump()))
    assert again.to_dict() == cfg.to_dict()


def test_method_nodes_declared():
    cfg = get_cfg()
    for n in METHOD_NODES:
        assert n in cfg


def test_mode_key_accepts_bool_from_command_line():
    """``RUNTIME.DOT_SINGLE_PASS False`` on the command line: a string mode key
    (default "auto") takes the boolean as "false" / "true"."""
    from mdistiller_ddp_amd.config import get_cfg
    cfg = get_cfg()
    cfg.merge_from_list(["RUNTIME.DOT_SINGLE_PASS", "False", "RUNTIME.TEACHER_LOOKAHEAD", "True"])
    assert cfg.RUNTIME.DOT_SINGLE_PASS == "false"
    assert cfg.RUNTIME.TEACHER_LOOKAHEAD == "true"
