"""CIFAR-100 / Tiny-ImageNet model registries (reference `models/cifar/__init__.py:22-80`).

``name -> (constructor, teacher_checkpoint_path | None)``.  Teacher checkpoints
are ``{"model": state_dict}`` files at
``<CKPT_ROOT>/cifar_teachers/<name>_vanilla/ckpt_epoch_240.pth``; CKPT_ROOT is
``$MDA_CKPT_ROOT`` or ``<repo>/download_ckpts``.
"""
import os

from .resnet import resnet8, resnet14, resnet20, resnet32, resnet44, resnet56, resnet110, resnet8x4, resnet32x4
from .resnetv2 import ResNet18, ResNet34, ResNet50, ResNet101, ResNet152
from .wrn import wrn_16_1, wrn_16_2, wrn_40_1, wrn_40_2
from .vgg import vgg19_bn, vgg16_bn, vgg13_bn, vgg11_bn, vgg8_bn
from .mobilenetv2 import mobile_half
from .shufflenet import ShuffleV1, ShuffleV2
from .mv2_tinyimagenet import mobilenetv2_tinyimagenet

_REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
CKPT_ROOT = os.environ.get("MDA_CKPT_ROOT", os.path.join(_REPO, "download_ckpts"))
cifar100_model_prefix = os.path.join(CKPT_ROOT, "cifar_teachers") + os.sep
tiny_imagenet_model_prefix = os.path.join(CKPT_ROOT, "tiny_imagenet_teachers") + os.sep


def _t(name):
    return cifar100_model_prefix + f"{name}_vanilla/ckpt_epoch_240.pth"


cifar_model_dict = {
    # teachers
    "resnet56": (resnet56, _t("resnet56")),
    "resnet110": (resnet110, _t("resnet110")),
    "resnet32x4": (resnet32x4, _t("resnet32x4")),
    "ResNet50": (ResNet50, _t("ResNet50")),
    "wrn_40_2": (wrn_40_2, _t("wrn_40_2")),
    "vgg13": (vgg13_bn, _t("vgg13")),
    # students
    "resnet8": (resnet8, None),
    "resnet14": (resnet14, None),
    "resnet20": (resnet20, None),
    "resnet32": (resnet32, None),
    "resnet44": (resnet44, None),
    "resnet8x4": (resnet8x4, None),
    "ResNet18": (ResNet18, None),
    "wrn_16_1": (wrn_16_1, None),
    "wrn_16_2": (wrn_16_2, None),
    "wrn_40_1": (wrn_40_1, None),
    "vgg8": (vgg8_bn, None),
    "vgg11": (vgg11_bn, None),
    "vgg16": (vgg16_bn, None),
    "vgg19": (vgg19_bn, None),
    "MobileNetV2": (mobile_half, None),
    "ShuffleV1": (ShuffleV1, None),
    "ShuffleV2": (ShuffleV2, None),
}

tiny_imagenet_model_dict = {
    "ResNet18": (ResNet18, tiny_imagenet_model_prefix + "ResNet18_vanilla/ti_res18"),
    "MobileNetV2": (mobilenetv2_tinyimagenet, None),
    "ShuffleV2": (ShuffleV2, None),
}
