"""Detection extras on CPU: deformable convolution (DCN v1/v2) against
regular-conv identities + gradcheck, the deformable ResNet stage, the dataset
evaluators (COCO / LVIS federated rules / Pascal VOC / semantic segmentation /
Cityscapes) on hand-checkable cases, and test-time augmentation."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mdistiller_ddp_amd.detection import evaluation as E
from mdistiller_ddp_amd.detection.deform import DeformConv, ModulatedDeformConv, deform_conv2d
from mdistiller_ddp_amd.detection.structures import Instances


# ----------------------------------------------------------------------------- deformable conv
@pytest.mark.parametrize("stride,pad,dil,groups,dg", [(1, 1, 1, 1, 1), (2, 1, 1, 2, 2), (1, 2, 2, 1, 4)])
def test_deform_zero_offset_is_conv(stride, pad, dil, groups, dg):
    torch.manual_seed(0)
    x = torch.randn(2, 8, 9, 11, dtype=torch.float64)
    w = torch.randn(6, 8 // groups, 3, 3, dtype=torch.float64)
    b = torch.randn(6, dtype=torch.float64)
    ref = F.conv2d(x, w, b, stride, pad, dil, groups)
    off = torch.zeros(2, dg * 18, *ref.shape[-2:], dtype=torch.float64)
    out = deform_conv2d(x, off, w, b, stride, pad, dil, groups, dg)
    torch.testing.assert_close(out, ref)
    mask = torch.full((2, dg * 9, *ref.shape[-2:]), 0.5, dtype=torch.float64)
    out2 = deform_conv2d(x, off, w, None, stride, pad, dil, groups, dg, mask=mask)
    torch.testing.assert_close(out2, 0.5 * F.conv2d(x, w, None, stride, pad, dil, groups))


def test_deform_integer_shift():
    torch.manual_seed(1)
    x = torch.randn(1, 4, 7, 7, dtype=torch.float64)
    w = torch.randn(5, 4, 3, 3, dtype=torch.float64)
    off = torch.zeros(1, 18, 7, 7, dtype=torch.float64)
    off[:, 0::2] = 1.0   # every tap samples one row lower (dy = +1)
    off[:, 1::2] = -2.0  # and two columns to the left
    out = deform_conv2d(x, off, w, None, 1, 1)
    # tap (a, b) of output (i, j) reads x[i - 1 + a + 1, j - 1 + b - 2] (zero outside x)
    xp = F.pad(x, (3, 3, 3, 3))
    torch.testing.assert_close(out, F.conv2d(xp[:, :, 3:3 + 7 + 2, 0:7 + 2], w))


def test_deform_gradcheck():
    torch.manual_seed(2)
    x = torch.randn(1, 4, 5, 5, dtype=torch.float64, requires_grad=True)
    w = torch.randn(4, 2, 3, 3, dtype=torch.float64, requires_grad=True)
    off = (0.3 + 0.4 * torch.rand(1, 2 * 18, 5, 5, dtype=torch.float64)) * torch.sign(torch.randn(1, 36, 5, 5))
    off.requires_grad_(True)
    mask = torch.rand(1, 2 * 9, 5, 5, dtype=torch.float64, requires_grad=True)
    fn = lambda x_, o_, w_, m_: deform_conv2d(x_, o_, w_, None, 1, 1, 1, 2, 2, mask=m_)
    assert torch.autograd.gradcheck(fn, (x, off, w, mask), eps=1e-6, atol=1e-5)


def test_deform_modules_and_stage():
    from mdistiller_ddp_amd.detection.backbone import (BottleneckBlock, DeformBottleneckBlock,
                                                       build_resnet_backbone)
    from mdistiller_ddp_amd.detection.config import get_det_cfg
    torch.manual_seed(3)
    dc = DeformConv(8, 8, 3, padding=1)
    mc = ModulatedDeformConv(8, 8, 3, padding=1, deformable_groups=2)
    x = torch.randn(1, 8, 6, 6)
    assert dc(x, torch.zeros(1, 18, 6, 6)).shape == (1, 8, 6, 6)
    assert mc(x, torch.zeros(1, 36, 6, 6), torch.ones(1, 18, 6, 6)).shape == (1, 8, 6, 6)
    # a fresh deformable block (zero offsets) computes what a bottleneck with the same weights does
    for modulated in (False, True):
        d = DeformBottleneckBlock(16, 32, bottleneck_channels=8, stride=2, norm="",
                                  deform_modulated=modulated).eval()
        p = BottleneckBlock(16, 32, bottleneck_channels=8, stride=2, norm="").eval()
        sd = {k: v for k, v in d.state_dict().items() if not k.startswith("conv2_offset")}
        if modulated:  # the zero-initialised mask is sigmoid(0) = 0.5 on every tap
            sd["conv2.weight"] = sd["conv2.weight"] * 0.5
        p.load_state_dict(sd)
        xi = torch.randn(2, 16, 9, 9)
        torch.testing.assert_close(d(xi), p(xi), atol=1e-5, rtol=1e-5)
    cfg = get_det_cfg()
    cfg.MODEL.RESNETS.DEPTH = 50
    cfg.MODEL.RESNETS.NORM = "BN"
    cfg.MODEL.RESNETS.OUT_FEATURES = ["res3"]
    cfg.MODEL.RESNETS.DEFORM_ON_PER_STAGE = [False, True, False, False]
    cfg.MODEL.RESNETS.DEFORM_MODULATED = True
    cfg.MODEL.BACKBONE.FREEZE_AT = 0
    bb = build_resnet_backbone(cfg.MODEL)
    assert isinstance(bb.res3[0], DeformBottleneckBlock)
    out = bb(torch.randn(1, 3, 64, 64))["res3"]
    out.float().mean().backward()
    assert bb.res3[0].conv2_offset.weight.grad is not None
    assert bb.res3[0].conv2.weight.grad.abs().sum() > 0


# ----------------------------------------------------------------------------- evaluators
def _img(boxes, classes, scores=None, **kw):
    d = {"boxes": np.asarray(boxes, dtype=np.float64).reshape(-1, 4),
         "classes": np.asarray(classes, dtype=np.int64)}
    if scores is not None:
        d["scores"] = np.asarray(scores, dtype=np.float64)
    d.update(kw)
    return d


def test_voc_metric():
    gts = [_img([[0, 0, 10, 10], [20, 20, 40, 40]], [0, 1], difficult=np.array([0, 1]))]
    perfect = [_img([[0, 0, 10, 10]], [0], [0.9])]
    r = E.voc_evaluate(perfect, gts, 2)
    assert r["AP50"] == pytest.approx(100.0)  # class 1 only has a difficult box: not scored
    # one FP above one TP on a single gt: precision 1/2 at recall 1 -> 11-point AP 0.5
    fp_first = [_img([[50, 50, 60, 60], [0, 0, 10, 10]], [0, 0], [0.9, 0.8])]
    assert E.voc_class_ap(fp_first, gts, 0, 0.5, True) == pytest.approx(0.5)
    # area metric: precision envelope 0.5 over recall [0, 1]
    assert E.voc_class_ap(fp_first, gts, 0, 0.5, False) == pytest.approx(0.5)
    # a detection on the difficult box is neither TP nor FP
    with_diff = [_img([[20, 20, 40, 40], [0, 0, 10, 10]], [1, 0], [0.95, 0.9])]
    assert E.voc_evaluate(with_diff, gts, 2)["AP50"] == pytest.approx(100.0)


def test_coco_evaluator_matches_engine():
    from mdistiller_ddp_amd.detection.engine import coco_evaluate
    rng = np.random.default_rng(0)
    gts, preds = [], []
    for i in range(6):
        n = rng.integers(1, 5)
        xy = rng.uniform(0, 200, (n, 2))
        wh = rng.uniform(10, 120, (n, 2))
        b = np.concatenate([xy, xy + wh], 1)
        c = rng.integers(0, 3, n)
        gts.append(_img(b, c))
        jit = b + rng.normal(0, 4, b.shape)
        preds.append(_img(np.concatenate([jit, b[:1] + 50]), np.concatenate([c, c[:1]]),
                          rng.uniform(0.1, 1, n + 1)))
    ref = coco_evaluate(preds, gts, 3)
    new = E.coco_instance_evaluate(preds, gts, 3)
    for k in ("AP", "AP50", "AP75"):
        assert new[k] == pytest.approx(ref[k], abs=1e-9)


def test_lvis_federated_rules():
    gts = [_img([[0, 0, 10, 10]], [0], neg_category_ids=[2], not_exhaustive_category_ids=[]),
           _img([[0, 0, 10, 10]], [1], neg_category_ids=[], not_exhaustive_category_ids=[1])]
    base = [_img([[0, 0, 10, 10]], [0], [0.9]), _img([[0, 0, 10, 10]], [1], [0.9])]
    r0 = E.lvis_evaluate(base, gts, 3)
    assert r0["AP"] == pytest.approx(100.0)
    # class 1 is not annotated (nor negative) on image 0: its detections there are not evaluated
    extra_unk = [_img([[0, 0, 10, 10], [30, 30, 40, 40]], [0, 1], [0.9, 0.95]), base[1]]
    assert E.lvis_evaluate(extra_unk, gts, 3)["AP"] == pytest.approx(100.0)
    # class 1 not exhaustively annotated on image 1: an unmatched class-1 detection is ignored
    extra_ne = [base[0], _img([[0, 0, 10, 10], [50, 50, 60, 60]], [1, 1], [0.9, 0.95])]
    assert E.lvis_evaluate(extra_ne, gts, 3)["AP"] == pytest.approx(100.0)
    # the same unmatched detection in an EXHAUSTIVE image counts as a false positive
    extra_fp = [_img([[0, 0, 10, 10], [50, 50, 60, 60]], [0, 0], [0.9, 0.95]), base[1]]
    assert E.lvis_evaluate(extra_fp, gts, 3)["AP"] < 100.0
    # frequency buckets
    r = E.lvis_evaluate(base, gts, 3, category_frequency={0: "f", 1: "r", 2: "c"})
    assert r["APf"] == pytest.approx(100.0) and r["APr"] == pytest.approx(100.0)


def test_semseg_metrics():
    gt = np.array([[0, 0, 1, 1], [2, 2, 255, 1]])
    pred = np.array([[0, 1, 1, 1], [2, 0, 0, 1]])
    conf = E.semseg_confusion(pred, gt, 3)
    r = E.semseg_metrics(conf)
    # class 0: tp 1, gt 2, pred 2 -> IoU 1/3; class 1: tp 3, gt 3, pred 4 -> 3/4; class 2: tp 1, gt 2, pred 1 -> 1/2
    assert r["IoU-0"] == pytest.approx(100 / 3)
    assert r["IoU-1"] == pytest.approx(75.0)
    assert r["IoU-2"] == pytest.approx(50.0)
    assert r["mIoU"] == pytest.approx((100 / 3 + 75 + 50) / 3)
    assert r["pACC"] == pytest.approx(5 / 7 * 100)  # the 255 pixel is ignored
    ev = E.build_evaluator("cityscapes_sem_seg", 19)
    ev.reset()
    lab = torch.randint(0, 19, (8, 8))
    logits = F.one_hot(lab, 19).permute(2, 0, 1).float()
    ev.process([{"sem_seg": lab}], [{"sem_seg": logits}])
    assert ev.evaluate()["sem_seg"]["mIoU"] == pytest.approx(100.0)


def test_instance_evaluators_protocol():
    H, W = 32, 48
    m = torch.zeros(2, H, W, dtype=torch.uint8)
    m[0, 2:10, 3:20] = 1
    m[1, 15:30, 25:45] = 1
    boxes = torch.tensor([[3., 2., 20., 10.], [25., 15., 45., 30.]])
    gt = Instances((H, W), gt_boxes=boxes, gt_classes=torch.tensor([0, 1]), gt_masks=m)
    x = {"instances": gt, "height": H, "width": W}
    pred = Instances((H, W), pred_boxes=boxes.clone(), scores=torch.tensor([0.9, 0.8]),
                     pred_classes=torch.tensor([0, 1]), pred_masks=m.float())
    for typ, key in (("coco", "bbox"), ("lvis", "bbox"), ("pascal_voc", "bbox"), ("cityscapes_instance", "segm")):
        ev = E.build_evaluator(typ, 2, mask_on=True)
        ev.reset()
        ev.process([x], [{"instances": pred}])
        res = ev.evaluate()
        assert res[key]["AP"] == pytest.approx(100.0), (typ, res)
    both = E.build_evaluator("coco", 2, mask_on=True)
    both.process([x], [{"instances": pred}])
    r = both.evaluate()
    assert r["segm"]["AP"] == pytest.approx(100.0) and r["bbox"]["AP"] == pytest.approx(100.0)
    pan = E.build_evaluator("coco_panoptic_seg", 2)
    assert isinstance(pan, E.DatasetEvaluators)
    with pytest.raises(NotImplementedError):
        E.build_evaluator("unknown", 2)


def test_tta_merges_augmentations():
    from mdistiller_ddp_amd.detection.config import get_det_cfg
    from mdistiller_ddp_amd.detection.tta import GeneralizedRCNNWithTTA

    class SquareFinder(torch.nn.Module):
        """Detects the bright square; boxes in original coordinates (as the real
        model's post-processing returns them)."""

        def forward(self, inputs):
            outs = []
            for x in inputs:
                img = x["image"].float()
                ys, xs = torch.nonzero(img[0] > 128, as_tuple=True)
                h, w = img.shape[-2:]
                sy, sx = x["height"] / h, x["width"] / w
                b = torch.tensor([[xs.min() * sx, ys.min() * sy, (xs.max() + 1) * sx, (ys.max() + 1) * sy]])
                outs.append({"instances": Instances((x["height"], x["width"]), pred_boxes=b,
                                                    scores=torch.tensor([0.9]),
                                                    pred_classes=torch.tensor([3]))})
            return outs

    cfg = get_det_cfg()
    cfg.TEST.AUG.MIN_SIZES = (40, 80)
    cfg.TEST.AUG.MAX_SIZE = 1000
    img = torch.zeros(3, 40, 60, dtype=torch.uint8)
    img[:, 10:20, 5:25] = 255  # off-centre: a flip that is not undone would move it
    tta = GeneralizedRCNNWithTTA(cfg, SquareFinder())
    out = tta([{"image": img, "height": 40, "width": 60}])[0]["instances"]
    assert len(out) == 1  # 4 augmentations merged by NMS
    torch.testing.assert_close(out.pred_boxes[0], torch.tensor([5., 10., 25., 20.]), atol=1.0, rtol=0)
