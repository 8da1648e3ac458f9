"""Detection config: the Detectron2 default keys the reference's detection
YAMLs rely on (`detection/configs/**`), plus ``add_distillation_cfg``
(`detection/model/config.py:4-26`: ``MODEL.MOBILENETV2``, ``KD.{TYPE, DKD,
REVIEWKD}`` and the ``TEACHER.*`` mirror of the default tree,
`config.py:29-637`).  Built on the framework's yacs-compatible CfgNode;
``_BASE_`` inheritance is resolved the way Detectron2's loader does
(:func:`merge_det_file`).  ``RUNTIME`` holds this framework's extensions.
"""
from __future__ import annotations

import os

import yaml

from ..config.cfgnode import CfgNode as CN


def _model_node() -> CN:
    M = CN()
    M.LOAD_PROPOSALS = False
    M.MASK_ON = False
    M.KEYPOINT_ON = False
    M.DEVICE = "cuda"
    M.META_ARCHITECTURE = "GeneralizedRCNN"
    M.WEIGHTS = ""
    M.PIXEL_MEAN = [103.530, 116.280, 123.675]
    M.PIXEL_STD = [1.0, 1.0, 1.0]
    M.BACKBONE = CN({"NAME": "build_resnet_backbone", "FREEZE_AT": 2})
    M.FPN = CN({"IN_FEATURES": [], "OUT_CHANNELS": 256, "NORM": "", "FUSE_TYPE": "sum"})
    M.PROPOSAL_GENERATOR = CN({"NAME": "RPN", "MIN_SIZE": 0})
    M.ANCHOR_GENERATOR = CN({"NAME": "DefaultAnchorGenerator", "SIZES": [[32, 64, 128, 256, 512]],
                             "ASPECT_RATIOS": [[0.5, 1.0, 2.0]], "ANGLES": [[-90, 0, 90]],
                             "OFFSET": 0.0})
    M.RPN = CN({"HEAD_NAME": "StandardRPNHead", "IN_FEATURES": ["res4"], "BOUNDARY_THRESH": -1,
                "IOU_THRESHOLDS": [0.3, 0.7], "IOU_LABELS": [0, -1, 1],
                "BATCH_SIZE_PER_IMAGE": 256, "POSITIVE_FRACTION": 0.5,
                "BBOX_REG_LOSS_TYPE": "smooth_l1", "BBOX_REG_LOSS_WEIGHT": 1.0,
                "BBOX_REG_WEIGHTS": (1.0, 1.0, 1.0, 1.0), "SMOOTH_L1_BETA": 0.0, "LOSS_WEIGHT": 1.0,
                "PRE_NMS_TOPK_TRAIN": 12000, "PRE_NMS_TOPK_TEST": 6000,
                "POST_NMS_TOPK_TRAIN": 2000, "POST_NMS_TOPK_TEST": 1000, "NMS_THRESH": 0.7,
                "CONV_DIMS": [-1]})
    M.ROI_HEADS = CN({"NAME": "Res5ROIHeads", "NUM_CLASSES": 80, "IN_FEATURES": ["res4"],
                      "IOU_THRESHOLDS": [0.5], "IOU_LABELS": [0, 1], "BATCH_SIZE_PER_IMAGE": 512,
                      "POSITIVE_FRACTION": 0.25, "SCORE_THRESH_TEST": 0.05, "NMS_THRESH_TEST": 0.5,
                      "PROPOSAL_APPEND_GT": True})
    M.ROI_BOX_HEAD = CN({"NAME": "", "BBOX_REG_LOSS_TYPE": "smooth_l1", "BBOX_REG_LOSS_WEIGHT": 1.0,
                         "BBOX_REG_WEIGHTS": (10.0, 10.0, 5.0, 5.0), "SMOOTH_L1_BETA": 0.0,
                         "POOLER_RESOLUTION": 14, "POOLER_SAMPLING_RATIO": 0,
                         "POOLER_TYPE": "ROIAlignV2", "NUM_FC": 0, "FC_DIM": 1024, "NUM_CONV": 0,
                         "CONV_DIM": 256, "NORM": "", "CLS_AGNOSTIC_BBOX_REG": False,
                         "TRAIN_ON_PRED_BOXES": False})
    M.ROI_BOX_CASCADE_HEAD = CN({"BBOX_REG_WEIGHTS": ((10.0, 10.0, 5.0, 5.0), (20.0, 20.0, 10.0, 10.0),
                                                      (30.0, 30.0, 15.0, 15.0)),
                                 "IOUS": (0.5, 0.6, 0.7)})
    M.ROI_MASK_HEAD = CN({"NAME": "MaskRCNNConvUpsampleHead", "POOLER_RESOLUTION": 14,
                          "POOLER_SAMPLING_RATIO": 0, "NUM_CONV": 0, "CONV_DIM": 256, "NORM": "",
                          "CLS_AGNOSTIC_MASK": False, "POOLER_TYPE": "ROIAlignV2"})
    M.ROI_KEYPOINT_HEAD = CN({"NAME": "KRCNNConvDeconvUpsampleHead", "POOLER_RESOLUTION": 14,
                              "POOLER_SAMPLING_RATIO": 0, "CONV_DIMS": tuple(512 for _ in range(8)),
                              "NUM_KEYPOINTS": 17, "MIN_KEYPOINTS_PER_IMAGE": 1,
                              "NORMALIZE_LOSS_BY_VISIBLE_KEYPOINTS": True, "LOSS_WEIGHT": 1.0,
                              "POOLER_TYPE": "ROIAlignV2"})
    M.SEM_SEG_HEAD = CN({"NAME": "SemSegFPNHead", "IN_FEATURES": ["p2", "p3", "p4", "p5"],
                         "IGNORE_VALUE": 255, "NUM_CLASSES": 54, "CONVS_DIM": 128,
                         "COMMON_STRIDE": 4, "NORM": "GN", "LOSS_WEIGHT": 1.0})
    M.PANOPTIC_FPN = CN({"INSTANCE_LOSS_WEIGHT": 1.0,
                         "COMBINE": {"ENABLED": True, "OVERLAP_THRESH": 0.5, "STUFF_AREA_LIMIT": 4096,
                                     "INSTANCES_CONFIDENCE_THRESH": 0.5}})
    M.RETINANET = CN({"NUM_CLASSES": 80, "IN_FEATURES": ["p3", "p4", "p5", "p6", "p7"], "NUM_CONVS": 4,
                      "IOU_THRESHOLDS": [0.4, 0.5], "IOU_LABELS": [0, -1, 1], "PRIOR_PROB": 0.01,
                      "SCORE_THRESH_TEST": 0.05, "TOPK_CANDIDATES_TEST": 1000, "NMS_THRESH_TEST": 0.5,
                      "BBOX_REG_WEIGHTS": (1.0, 1.0, 1.0, 1.0), "FOCAL_LOSS_GAMMA": 2.0,
                      "FOCAL_LOSS_ALPHA": 0.25, "SMOOTH_L1_LOSS_BETA": 0.1,
                      "BBOX_REG_LOSS_TYPE": "smooth_l1", "NORM": ""})
    M.RESNETS = CN({"DEPTH": 50, "OUT_FEATURES": ["res4"], "NUM_GROUPS": 1, "NORM": "FrozenBN",
                    "WIDTH_PER_GROUP": 64, "STRIDE_IN_1X1": True, "RES5_DILATION": 1,
                    "RES2_OUT_CHANNELS": 256, "STEM_OUT_CHANNELS": 64,
                    "DEFORM_ON_PER_STAGE": [False, False, False, False], "DEFORM_MODULATED": False,
                    "DEFORM_NUM_GROUPS": 1})
    M.MOBILENETV2 = CN({"DEBUG": 0, "OUT_FEATURES": ["m2"], "NORM": "FrozenBN"})
    return M


def _input_node() -> CN:
    return CN({"MIN_SIZE_TRAIN": (800,), "MIN_SIZE_TRAIN_SAMPLING": "choice", "MAX_SIZE_TRAIN": 1333,
               "MIN_SIZE_TEST": 800, "MAX_SIZE_TEST": 1333, "RANDOM_FLIP": "horizontal",
               "CROP": {"ENABLED": False, "TYPE": "relative_range", "SIZE": [0.9, 0.9]},
               "FORMAT": "BGR", "MASK_FORMAT": "polygon"})


def _datasets_node() -> CN:
    return CN({"TRAIN": (), "PROPOSAL_FILES_TRAIN": (), "PRECOMPUTED_PROPOSAL_TOPK_TRAIN": 2000,
               "TEST": (), "PROPOSAL_FILES_TEST": (), "PRECOMPUTED_PROPOSAL_TOPK_TEST": 1000})


def _dataloader_node() -> CN:
    return CN({"NUM_WORKERS": 4, "ASPECT_RATIO_GROUPING": True, "SAMPLER_TRAIN": "TrainingSampler",
               "REPEAT_THRESHOLD": 0.0, "FILTER_EMPTY_ANNOTATIONS": True})


def _solver_node() -> CN:
    return CN({"LR_SCHEDULER_NAME": "WarmupMultiStepLR", "MAX_ITER": 40000, "BASE_LR": 0.001,
               "MOMENTUM": 0.9, "NESTEROV": False, "WEIGHT_DECAY": 0.0001, "WEIGHT_DECAY_NORM": 0.0,
               "GAMMA": 0.1, "STEPS": (30000,), "WARMUP_FACTOR": 1.0 / 1000, "WARMUP_ITERS": 1000,
               "WARMUP_METHOD": "linear", "CHECKPOINT_PERIOD": 5000, "IMS_PER_BATCH": 16,
               "REFERENCE_WORLD_SIZE": 0, "BIAS_LR_FACTOR": 1.0, "WEIGHT_DECAY_BIAS": 0.0001,
               "CLIP_GRADIENTS": {"ENABLED": False, "CLIP_TYPE": "value", "CLIP_VALUE": 1.0,
                                  "NORM_TYPE": 2.0},
               "AMP": {"ENABLED": False}})


def _test_node() -> CN:
    return CN({"EXPECTED_RESULTS": [], "EVAL_PERIOD": 0, "KEYPOINT_OKS_SIGMAS": [],
               "DETECTIONS_PER_IMAGE": 100,
               "AUG": {"ENABLED": False, "MIN_SIZES": (400, 500, 600, 700, 800, 900, 1000, 1100, 1200),
                       "MAX_SIZE": 4000, "FLIP": True},
               "PRECISE_BN": {"ENABLED": False, "NUM_ITER": 200}})


def _misc(node: CN) -> None:
    node.OUTPUT_DIR = "./output"
    node.SEED = -1
    node.CUDNN_BENCHMARK = False
    node.VIS_PERIOD = 0
    node.GLOBAL = CN({"HACK": 1.0})


def add_teacher_cfg(cfg: CN) -> None:
    """``cfg.TEACHER``: a full mirror of the default tree (reference `config.py:29-637`)."""
    T = CN()
    T.KD = CN({"FEATURE_KD_MASK": "None"})
    T.MODEL = _model_node()
    T.INPUT = _input_node()
    T.DATASETS = _datasets_node()
    T.DATALOADER = _dataloader_node()
    T.SOLVER = _solver_node()
    T.TEST = _test_node()
    _misc(T)
    cfg.TEACHER = T


def add_distillation_cfg(cfg: CN) -> None:
    """Reference `detection/model/config.py:4-26`."""
    cfg.MODEL.MOBILENETV2 = CN({"DEBUG": 0, "OUT_FEATURES": ["m2"], "NORM": "FrozenBN"})
    cfg.KD = CN({"TYPE": "DKD", "DKD": {"ALPHA": 1.0, "BETA": 0.25, "T": 1.0},
                 "REVIEWKD": {"LOSS_WEIGHT": 1.0}})
    add_teacher_cfg(cfg)


def get_det_cfg() -> CN:
    """A fresh default detection config (Detectron2 defaults + distillation keys)."""
    C = CN()
    C.VERSION = 2
    C.MODEL = _model_node()
    C.INPUT = _input_node()
    C.DATASETS = _datasets_node()
    C.DATALOADER = _dataloader_node()
    C.SOLVER = _solver_node()
    C.TEST = _test_node()
    _misc(C)
    # framework extensions (not in the reference)
    C.RUNTIME = CN({
        "BACKEND": "auto",          # auto | hip | torch
        "DTYPE": "bf16",            # bf16 autocast on GPU | fp32
        "TEACHER_STREAM": True,     # teacher backbone on its own HIP stream
        "BUCKET_MB": 16.0,          # gradient all-reduce bucket size
        "LOG_PERIOD": 20,
        "SYNTHETIC": True,          # COCO-shaped synthetic data (no dataset in this image)
        "SYNTHETIC_SIZE": (0, 0),   # fixed (H, W) of synthetic images; (0, 0) = INPUT sizes
        "SYNTHETIC_VAL_IMAGES": 16,
        "COCO_JSON": "",            # COCO-format instances json (+ COCO_IMAGE_ROOT) instead
        "COCO_IMAGE_ROOT": "",
        "RANDOM_INIT_DAMP": 0.25,   # residual-branch damping when no MODEL.WEIGHTS is loaded
        # evaluator_type of the test set (the reference reads it from the
        # dataset metadata): coco | lvis | pascal_voc | cityscapes_instance |
        # cityscapes_sem_seg | sem_seg | coco_panoptic_seg
        "EVALUATOR_TYPE": "coco",
    })
    add_distillation_cfg(C)
    return C


def merge_det_file(cfg: CN, path: str) -> None:
    """``cfg.merge_from_file`` with Detectron2's ``_BASE_`` inheritance."""
    with open(path, "r") as f:
        data = yaml.safe_load(f) or {}
    base = data.pop("_BASE_", None)
    if base is not None:
        if not os.path.isabs(base):
            base = os.path.join(os.path.dirname(path), base)
        merge_det_file(cfg, base)
    cfg.merge_from_other_cfg(CN(data))
