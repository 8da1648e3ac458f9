"""Training engine (reference `mdistiller/engine/`)."""
from .trainer import trainer_dict, BaseTrainer, CRDTrainer, DOT, CRDDOT
from .step import TrainStep, DeviceMeters
from .optim import FlatParams, FlatSGD, FlatAdam, FlatDOT, build_optimizer
from .utils import (AverageMeter, accuracy, adjust_learning_rate, validate, save_checkpoint,
                    load_checkpoint, log_msg)
from .build import build_distiller, build_teacher, build_student

__all__ = ["trainer_dict", "BaseTrainer", "CRDTrainer", "DOT", "CRDDOT", "TrainStep",
           "DeviceMeters", "FlatParams", "FlatSGD", "FlatAdam", "FlatDOT", "build_optimizer",
           "AverageMeter", "accuracy", "adjust_learning_rate", "validate", "save_checkpoint",
           "load_checkpoint", "log_msg", "build_distiller", "build_teacher", "build_student"]
