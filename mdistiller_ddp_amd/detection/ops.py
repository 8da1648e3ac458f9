"""Detection kernels: ROIAlign over every FPN level in one launch, and NMS
(``ops/csrc/det.hip``; the reference's detectors get both from Detectron2's
CUDA extension -- SURVEY K17).  Each has an fp32 PyTorch reference that is
the CPU path and the numerical oracle of the GPU tests.

Semantics: Detectron2 ``ROIAlignV2`` (``aligned=True``: pixel model shifted
by -0.5; ``sampling_ratio <= 0``: an adaptive ceil(roi / bin) grid per bin;
samples outside the map contribute zero) and torchvision NMS (a box is
suppressed by a higher-scoring kept box with IoU > threshold).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import _ext
from ..ops.backend import hip_enabled_for

_MAX_LEVELS = 5


# ----------------------------------------------------------------------------- ROIAlign
def _axis_weights(start, bin_size, grid, n_bins, size, gmax):
    """``[R, n_bins, size]``: summed bilinear weights of one axis' valid samples.

    Bilinear sampling and the out-of-map rule are separable, so a 2-D RoI
    bin is ``Ay @ X @ Ax^T`` with these per-axis weight matrices.
    """
    R = start.shape[0]
    dev = start.device
    p = torch.arange(n_bins, device=dev, dtype=torch.float32).view(1, -1, 1)
    g = torch.arange(gmax, device=dev, dtype=torch.float32).view(1, 1, -1)
    gr = grid.clamp(min=1).to(torch.float32).view(-1, 1, 1)
    b = bin_size.view(-1, 1, 1)
    coord = start.view(-1, 1, 1) + p * b + (g + 0.5) * b / gr
    valid = (g < grid.view(-1, 1, 1).to(torch.float32)) & (coord >= -1.0) & (coord <= float(size))
    c = coord.clamp(min=0.0)
    lo = c.floor().to(torch.int64)
    at_end = lo >= size - 1
    lo = torch.where(at_end, torch.full_like(lo, size - 1), lo)
    hi = torch.where(at_end, lo, lo + 1)
    c = torch.where(at_end, lo.to(c.dtype), c)
    frac = c - lo.to(c.dtype)
    vf = valid.to(c.dtype)
    A = torch.zeros(R, n_bins, size, device=dev, dtype=torch.float32)
    A.scatter_add_(2, lo, (1.0 - frac) * vf)
    A.scatter_add_(2, hi, frac * vf)
    return A


def roi_align_ref(x, rois, output_size, spatial_scale, sampling_ratio=0, aligned=True):
    """fp32 PyTorch ROIAlign; ``x`` [N, C, H, W], ``rois`` [R, 5] (batch, x1, y1, x2, y2)."""
    PH, PW = output_size
    N, C, H, W = x.shape
    R = rois.shape[0]
    if R == 0:
        return x.new_zeros((0, C, PH, PW))
    r = rois.to(torch.float32)
    off = 0.5 if aligned else 0.0
    x1 = r[:, 1] * spatial_scale - off
    y1 = r[:, 2] * spatial_scale - off
    rw = r[:, 3] * spatial_scale - off - x1
    rh = r[:, 4] * spatial_scale - off - y1
    if not aligned:
        rw = rw.clamp(min=1.0)
        rh = rh.clamp(min=1.0)
    bw, bh = rw / PW, rh / PH
    if sampling_ratio > 0:
        gh = torch.full((R,), int(sampling_ratio), dtype=torch.int64, device=r.device)
        gw = gh.clone()
    else:
        gh = torch.ceil(rh / PH).to(torch.int64).clamp(min=0)
        gw = torch.ceil(rw / PW).to(torch.int64).clamp(min=0)
    ay = _axis_weights(y1, bh, gh, PH, H, max(int(gh.max()), 1))
    ax = _axis_weights(x1, bw, gw, PW, W, max(int(gw.max()), 1))
    ay = ay / (gh * gw).clamp(min=1).to(torch.float32).view(-1, 1, 1)
    xf = x.to(torch.float32)
    bidx = r[:, 0].to(torch.int64)
    out = xf.new_zeros((R, C, PH, PW))
    for b in range(N):
        sel = torch.nonzero(bidx == b, as_tuple=True)[0]
        for s in range(0, sel.numel(), 64):
            i = sel[s:s + 64]
            t = torch.einsum("rph,chw->rcpw", ay[i], xf[b])
            out = out.index_copy(0, i, torch.einsum("rcpw,rqw->rcpq", t, ax[i]))
    return out.to(x.dtype)


def multilevel_roi_align_ref(xs, rois, levels, output_size, scales, sampling_ratio=0, aligned=True):
    if len(xs) == 1:
        return roi_align_ref(xs[0], rois, output_size, scales[0], sampling_ratio, aligned)
    R, C = rois.shape[0], xs[0].shape[1]
    out = xs[0].new_zeros((R, C) + tuple(output_size), dtype=torch.float32)
    for l, (x, s) in enumerate(zip(xs, scales)):
        idx = torch.nonzero(levels == l, as_tuple=True)[0]
        if idx.numel():
            part = roi_align_ref(x, rois[idx], output_size, s, sampling_ratio, aligned)
            out = out.index_copy(0, idx, part.to(torch.float32))
    return out.to(xs[0].dtype)


def _native_ok(xs) -> bool:
    x0 = xs[0]
    if not (hip_enabled_for(x0) and 1 <= len(xs) <= _MAX_LEVELS):
        return False
    return all(x.dim() == 4 and x.dtype == x0.dtype and x.dtype in (torch.float32, torch.bfloat16)
               and x.shape[:2] == x0.shape[:2] and x.device == x0.device for x in xs)


def _level_tables(ptrs, hw, scales):
    return (torch.tensor(ptrs, dtype=torch.int64),
            torch.tensor([int(v) for s in hw for v in s], dtype=torch.int64),
            torch.tensor([float(s) for s in scales], dtype=torch.float32))


class _ROIAlignHIP(torch.autograd.Function):
    """Multi-level ROIAlign on ``mda_roi_align_{fwd,bwd}`` (NHWC in and out)."""

    @staticmethod
    def forward(ctx, rois, levels, output_size, scales, sampling_ratio, aligned, *xs):
        PH, PW = output_size
        x0 = xs[0]
        dt = 0 if x0.dtype == torch.float32 else 1
        xc = [x.contiguous(memory_format=torch.channels_last) for x in xs]
        C = x0.shape[1]
        R = rois.shape[0]
        out = torch.empty((R, C, PH, PW), dtype=x0.dtype, device=x0.device,
                          memory_format=torch.channels_last)
        ptrs, dims, sc = _level_tables([x.data_ptr() for x in xc], [x.shape[2:] for x in xc], scales)
        _ext.call("mda_roi_align_fwd", dt, len(xc), ptrs, dims, sc, rois, levels, out, R, C, PH, PW,
                  int(sampling_ratio), int(aligned))
        ctx.save_for_backward(rois, levels)
        ctx.meta = (PH, PW, tuple(scales), int(sampling_ratio), int(aligned),
                    [tuple(x.shape) for x in xs], x0.dtype, dt)
        return out

    @staticmethod
    def backward(ctx, dout):
        rois, levels = ctx.saved_tensors
        PH, PW, scales, sampling, aligned, shapes, dtype, dt = ctx.meta
        need = ctx.needs_input_grad[6:]
        if not any(need):
            return (None,) * (6 + len(shapes))
        dout = dout.to(dtype).contiguous(memory_format=torch.channels_last)
        dxs = [torch.zeros((n, h, w, c), dtype=torch.float32, device=dout.device)
               for (n, c, h, w) in shapes]
        ptrs, dims, sc = _level_tables([d.data_ptr() for d in dxs], [(s[2], s[3]) for s in shapes],
                                       scales)
        _ext.call("mda_roi_align_bwd", dt, len(dxs), ptrs, dims, sc, rois, levels, dout,
                  rois.shape[0], shapes[0][1], PH, PW, sampling, aligned)
        grads = [d.permute(0, 3, 1, 2).to(dtype) if n else None for d, n in zip(dxs, need)]
        return (None,) * 6 + tuple(grads)


def multilevel_roi_align(xs, rois, levels, output_size, scales, sampling_ratio=0, aligned=True):
    """Pool ``rois`` [R, 5] from ``xs[levels[r]]`` (scale ``scales[level]``) -> [R, C, PH, PW]."""
    output_size = tuple(int(v) for v in output_size)
    if rois.shape[0] == 0:
        return xs[0].new_zeros((0, xs[0].shape[1]) + output_size)
    if _native_ok(xs):
        r = rois.to(torch.float32).contiguous()
        lv = levels.to(torch.int32).contiguous() if (levels is not None and len(xs) > 1) else None
        return _ROIAlignHIP.apply(r, lv, output_size, list(scales), int(sampling_ratio),
                                  bool(aligned), *xs)
    return multilevel_roi_align_ref(xs, rois, levels, output_size, scales, sampling_ratio, aligned)


def roi_align(x, rois, output_size, spatial_scale, sampling_ratio=0, aligned=True):
    return multilevel_roi_align([x], rois, None, output_size, [spatial_scale], sampling_ratio,
                                aligned)


# ----------------------------------------------------------------------------- NMS
def nms_ref(boxes, scores, iou_threshold, max_keep=-1):
    """Greedy NMS on the host; returns kept indices in descending-score order."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    order = torch.argsort(scores.detach().float(), descending=True)
    b = boxes.detach()[order].double().cpu().numpy()
    n = b.shape[0]
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    sup = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if sup[i]:
            continue
        keep.append(i)
        if 0 < max_keep <= len(keep):
            break
        xx1 = np.maximum(b[i, 0], b[i + 1:, 0])
        yy1 = np.maximum(b[i, 1], b[i + 1:, 1])
        xx2 = np.minimum(b[i, 2], b[i + 1:, 2])
        yy2 = np.minimum(b[i, 3], b[i + 1:, 3])
        inter = np.clip(xx2 - xx1, 0, None) * np.clip(yy2 - yy1, 0, None)
        union = area[i] + area[i + 1:] - inter
        iou = np.where(inter > 0, inter / np.where(union > 0, union, 1.0), 0.0)
        sup[i + 1:] |= iou > iou_threshold
    return order[torch.as_tensor(keep, dtype=torch.int64, device=order.device)]


def nms(boxes, scores, iou_threshold, max_keep=-1):
    """Kept indices (descending score), at most ``max_keep`` when > 0."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    n = boxes.shape[0]
    if hip_enabled_for(boxes) and n <= 500_000:
        order = torch.argsort(scores.detach().float(), descending=True)
        b = boxes.detach()[order].to(torch.float32).contiguous()
        nblk = (n + 63) // 64
        mask = torch.empty(n * nblk, dtype=torch.int64, device=b.device)
        keep = torch.empty(n, dtype=torch.uint8, device=b.device)
        cnt = torch.empty(1, dtype=torch.int32, device=b.device)
        _ext.call("mda_nms", b, n, float(iou_threshold), mask, int(max_keep), keep, cnt)
        return order[keep.bool()]
    return nms_ref(boxes, scores, iou_threshold, max_keep)


def batched_nms(boxes, scores, idxs, iou_threshold, max_keep=-1):
    """NMS within each ``idxs`` group (coordinate-offset trick: one launch)."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    b = boxes.float()
    off = idxs.to(b.dtype) * (b.max() + 1)
    return nms(b + off[:, None], scores, iou_threshold, max_keep)
