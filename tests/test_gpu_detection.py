"""Detection HIP kernels (csrc/det.hip) vs the fp32 PyTorch references:
multi-level ROIAlign forward/backward over NHWC fp32 and bf16 maps (aligned
and legacy pixel models, adaptive and fixed sampling grids) and the
wave64-ballot NMS (plain, capped, batched)."""
import pytest
import torch

from mdistiller_ddp_amd.detection import ops as O
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand_rois(R, N, img_h, img_w, g):
    x1 = torch.rand(R, generator=g) * img_w * 0.9 - 4
    y1 = torch.rand(R, generator=g) * img_h * 0.9 - 4
    bw = torch.rand(R, generator=g) * img_w * 0.5 + 0.5
    bh = torch.rand(R, generator=g) * img_h * 0.5 + 0.5
    b = torch.randint(0, N, (R,), generator=g).float()
    return torch.stack([b, x1, y1, x1 + bw, y1 + bh], 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("aligned,sampling", [(True, 0), (False, 2), (True, 2)])
@pytest.mark.parametrize("C", [64, 256])
def test_roi_align_multilevel(dtype, aligned, sampling, C):
    g = torch.Generator().manual_seed(0)
    N, img_h, img_w = 2, 128, 192
    scales = [1 / 4, 1 / 8, 1 / 16, 1 / 32]
    xs = [torch.randn(N, C, int(img_h * s), int(img_w * s), generator=g) for s in scales]
    R = 300
    rois = _rand_rois(R, N, img_h, img_w, g).to(DEV)
    levels = torch.randint(0, 4, (R,), generator=g).to(torch.int32).to(DEV)
    xh = [x.to(DEV).to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
          for x in xs]
    with use_backend("hip"):
        out = O.multilevel_roi_align(xh, rois, levels, (7, 7), scales, sampling, aligned)
    gout = torch.randn(out.shape, generator=g).to(DEV)
    out.float().backward(gout)
    xr = [x.to(dtype).float().to(DEV).requires_grad_(True) for x in xs]
    with use_backend("torch"):
        ref = O.multilevel_roi_align(xr, rois, levels, (7, 7), scales, sampling, aligned)
    ref.backward(gout)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref.detach(), atol=tol, rtol=tol)
    for a, b in zip(xh, xr):
        rel = ((a.grad.float() - b.grad).norm() / (b.grad.norm() + 1e-12)).item()
        assert rel < (1e-4 if dtype == torch.float32 else 1e-2), rel


def test_roi_align_single_level_mask_targets():
    """C = 1 crop-and-resize of bit masks (the Mask R-CNN target path)."""
    g = torch.Generator().manual_seed(1)
    m = (torch.rand(5, 1, 60, 80, generator=g) > 0.5).float()
    rois = torch.cat([torch.arange(5).float()[:, None], _rand_rois(5, 1, 60, 80, g)[:, 1:]], 1)
    with use_backend("hip"):
        a = O.roi_align(m.to(DEV), rois.to(DEV), (28, 28), 1.0, 0, True)
    b = O.roi_align_ref(m, rois, (28, 28), 1.0, 0, True)
    torch.testing.assert_close(a.cpu(), b, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 700, 5000])
def test_nms_matches_reference(n):
    g = torch.Generator().manual_seed(n)
    xy = torch.rand(n, 2, generator=g) * 500
    wh = torch.rand(n, 2, generator=g) * 80 + 1
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(n, generator=g)
    ref = O.nms_ref(boxes, scores, 0.5)
    with use_backend("hip"):
        k = O.nms(boxes.to(DEV), scores.to(DEV), 0.5)
        k10 = O.nms(boxes.to(DEV), scores.to(DEV), 0.5, max_keep=10)
        cls = torch.randint(0, 3, (n,), generator=g)
        kb = O.batched_nms(boxes.to(DEV), scores.to(DEV), cls.to(DEV), 0.6)
    assert torch.equal(k.cpu(), ref)
    assert torch.equal(k10.cpu(), ref[:10])
    off = cls.float() * (boxes.max() + 1)
    assert torch.equal(kb.cpu(), O.nms_ref(boxes + off[:, None], scores, 0.6))


@pytest.mark.parametrize("path", ["DKD/DKD-R18-R101.yaml", "ReviewKD/ReviewKD-R18-R101-Mask.yaml"])
def test_rcnnkd_gpu_train_steps(path):
    """Three bf16 training steps of the distilled detector on the GPU
    (HIP ROIAlign / NMS / fused DKD on the hot path): finite losses, the
    student moves, the teacher does not."""
    import os
    from mdistiller_ddp_amd.detection.data import build_detection_data
    from mdistiller_ddp_amd.detection.engine import DetectionTrainer
    from mdistiller_ddp_amd.detection.rcnn import build_model
    from tests.test_detection_cpu import tiny_cfg
    torch.manual_seed(0)
    cfg = tiny_cfg(path)
    cfg.RUNTIME.SYNTHETIC_SIZE = (256, 320)
    dev = torch.device(DEV)
    model = build_model(cfg).to(dev)
    _, loader = build_detection_data(cfg, device=dev)
    tr = DetectionTrainer(cfg, model, loader, dev)
    t0 = {k: v.clone() for k, v in model.teacher.state_dict().items()}
    s0 = tr.flat.data.clone()
    it = iter(loader)
    with use_backend("hip"):
        for _ in range(3):
            total, losses = tr.run_step(next(it))
            for k, v in losses.items():
                assert torch.isfinite(v).item(), (k, float(v))
    torch.cuda.synchronize()
    assert (tr.flat.data - s0).abs().max() > 0
    for k, v in model.teacher.state_dict().items():
        assert torch.equal(v, t0[k]), k
