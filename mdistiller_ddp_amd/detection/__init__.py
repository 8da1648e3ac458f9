"""Detection distillation side tree (reference `detection/`): Faster/Mask
R-CNN students distilled from a frozen teacher with DKD on ROI logits and/or
ReviewKD on FPN features, on HIP ROIAlign / NMS kernels (``ops/csrc/det.hip``)."""
from .config import get_det_cfg, merge_det_file  # noqa: F401
from .rcnn import RCNNKD, GeneralizedRCNN, build_model  # noqa: F401
