from .cifar import cifar_model_dict, tiny_imagenet_model_dict
from .imagenet import imagenet_model_dict
from ._base import ModelBase, Lambda, check_staged_forward, run_staged


def build_model(dataset: str, name: str, num_classes: int, pretrained: bool = False):
    """Construct a zoo model by (dataset type, registry name)."""
    if dataset == "imagenet":
        return imagenet_model_dict[name](pretrained=pretrained, num_classes=num_classes)
    table = tiny_imagenet_model_dict if dataset == "tiny_imagenet" else cifar_model_dict
    ctor, _ = table[name]
    return ctor(num_classes=num_classes)


def teacher_ckpt_path(dataset: str, name: str):
    if dataset == "imagenet":
        return None
    table = tiny_imagenet_model_dict if dataset == "tiny_imagenet" else cifar_model_dict
    return table[name][1]
