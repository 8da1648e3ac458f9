"""Model / distiller construction from a cfg (reference `tools/train.py:46-97`)."""
from __future__ import annotations

import os

import torch

from ..models import build_model, teacher_ckpt_path
from ..models.imagenet import imagenet_model_dict
from ..distillers import distiller_dict, Vanilla
from ..utils.logging import log_msg, master_print

NUM_CLASSES = {"cifar100": 100, "imagenet": 1000, "tiny_imagenet": 200}


def load_checkpoint(path: str, map_location="cpu"):
    """Checkpoints written by this framework (and the reference's teacher
    ``{"model": state_dict}`` files) load with ``weights_only=True``."""
    with open(path, "rb") as f:
        return torch.load(f, map_location=map_location, weights_only=True)


def build_teacher(cfg, num_classes: int):
    ds = cfg.DATASET.TYPE
    name = cfg.DISTILLER.TEACHER
    if ds == "imagenet":
        pretrained = not cfg.DISTILLER.RANDOM_TEACHER and not cfg.DISTILLER.TEACHER_CKPT
        try:
            model = imagenet_model_dict[name](pretrained=pretrained, num_classes=num_classes)
        except (FileNotFoundError, RuntimeError, OSError) as e:
            if not cfg.DISTILLER.RANDOM_TEACHER:
                raise
            master_print(log_msg(f"teacher {name}: {e}; using random init", "WARN"))
            model = imagenet_model_dict[name](pretrained=False, num_classes=num_classes)
        path = cfg.DISTILLER.TEACHER_CKPT or None
    else:
        model = build_model(ds, name, num_classes)
        path = cfg.DISTILLER.TEACHER_CKPT or teacher_ckpt_path(ds, name)
    if path and os.path.exists(path):
        sd = load_checkpoint(path)
        sd = sd.get("model", sd)
        model.load_state_dict(sd)
    elif ds != "imagenet" or cfg.DISTILLER.TEACHER_CKPT:
        if not cfg.DISTILLER.RANDOM_TEACHER:
            raise FileNotFoundError(
                f"teacher checkpoint not found: {path} (set DISTILLER.RANDOM_TEACHER True "
                "to benchmark with a random-init teacher)")
        master_print(log_msg(f"teacher {name}: checkpoint {path} missing; random init", "WARN"))
    return model


def build_student(cfg, num_classes: int):
    ds = cfg.DATASET.TYPE
    if ds == "imagenet":
        return imagenet_model_dict[cfg.DISTILLER.STUDENT](pretrained=False, num_classes=num_classes)
    return build_model(ds, cfg.DISTILLER.STUDENT, num_classes)


def build_distiller(cfg, num_classes: int = None, device="cpu", num_data: int = 0):
    num_classes = num_classes or NUM_CLASSES[cfg.DATASET.TYPE]
    student = build_student(cfg, num_classes)
    typ = cfg.DISTILLER.TYPE
    if typ == "NONE":
        distiller = Vanilla(student)
    else:
        teacher = build_teacher(cfg, num_classes)
        cls = distiller_dict[typ]
        if typ == "CRD":
            distiller = cls(student, teacher, cfg, num_data)
        else:
            distiller = cls(student, teacher, cfg)
    return distiller.to(device)
