"""HIP paths of the fused layer ops (``ops/nn.py``).

Inference-mode conv+BN(+residual)(+act) -- every teacher layer, and the
student during validation -- runs as ONE launch of the MFMA implicit-GEMM
kernel (``csrc/conv_igemm.hip``) with BN folded into the packed bf16 weights
and a per-channel bias.  Packing/folding happens once per weight version
(the frozen teacher: once per run) and is cached on the module.

Activations on this path are bf16 NHWC (``torch.channels_last``) end to end.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _ext

_ACT = {"none": 0, "relu": 1, "relu6": 2}


def _autocast_bf16() -> bool:
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


def _needs_grad(x, conv, bn) -> bool:
    if not torch.is_grad_enabled():
        return False
    if x.requires_grad or conv.weight.requires_grad:
        return True
    if bn is not None and bn.weight is not None and bn.weight.requires_grad:
        return True
    return False


# RUNTIME.FOLD_TEACHER_BN: fold frozen BN into the packed conv weights (one
# launch per teacher layer).  Off = conv kernel without BN, then PyTorch BN
# (A/B and debugging only).
_FOLD = {"on": True}


def set_fold_bn(flag: bool) -> None:
    _FOLD["on"] = bool(flag)


def conv_supported(x, conv, bn) -> bool:
    if not (x.is_cuda and x.dim() == 4 and isinstance(conv, nn.Conv2d)):
        return False
    if bn is not None and not _FOLD["on"]:
        return False
    if conv.groups != 1:
        from .hip_train import dw_supported_geometry
        if not dw_supported_geometry(conv):
            return False
    if conv.dilation != (1, 1) or conv.padding_mode != "zeros":
        return False
    if conv.stride[0] != conv.stride[1] or not isinstance(conv.padding, tuple):
        return False
    if conv.padding[0] != conv.padding[1]:
        return False
    if bn is not None and (bn.training or not bn.track_running_stats):
        return False
    if x.dtype == torch.bfloat16:
        pass
    elif not _autocast_bf16():
        return False
    return not _needs_grad(x, conv, bn)


def bn_supported(x, bn) -> bool:
    """Inference BN (+res) (+act) on an existing activation: frozen statistics
    -> per-channel scale/shift (cached per version), one ``mda_bn_apply``."""
    if not (x.is_cuda and x.dim() == 4 and isinstance(bn, nn.BatchNorm2d)):
        return False
    if bn.training or not bn.track_running_stats or x.shape[1] % 8:
        return False
    if torch.is_grad_enabled() and (x.requires_grad or (bn.weight is not None and bn.weight.requires_grad)):
        return False
    return x.dtype == torch.bfloat16 or _autocast_bf16()


@torch.no_grad()
def _bn_affine(bn):
    key = tuple(t._version for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var)
                if t is not None)
    if bn.weight is not None and bn.weight.requires_grad:
        key = key + (("gen", _GEN[0]),)
    cache = getattr(bn, "_mda_affine", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    C = bn.running_mean.numel()
    dev = bn.running_mean.device
    g = bn.weight.float() if bn.weight is not None else torch.ones(C, device=dev)
    b = bn.bias.float() if bn.bias is not None else torch.zeros(C, device=dev)
    sc = (g / torch.sqrt(bn.running_var.float() + bn.eps)).contiguous()
    sh = (b - bn.running_mean.float() * sc).contiguous()
    bn._mda_affine = (key, sc, sh)
    return sc, sh


def bn_act(x, bn, act, residual, want_preact):
    sc, sh = _bn_affine(bn)
    x = _nhwc_bf16(x)
    N, C, H, W = x.shape
    out = torch.empty_like(x)
    pre = torch.empty_like(x) if want_preact else None
    res = _nhwc_bf16(residual) if residual is not None else None
    _ext.call("mda_bn_apply", x, sc, sh, res, out, pre, N * H * W, C, _ACT[act])
    return out, pre


# Bumped by every training step (and checkpoint load): the native optimizer
# and BN-statistics kernels write parameters / running stats through raw
# pointers, which does not advance ``Tensor._version``, so the packed-weight
# caches of TRAINABLE layers are keyed on this generation as well.  Frozen
# layers (the teacher) keep their pack for the whole run.
_GEN = [0]


def bump_weight_generation() -> None:
    _GEN[0] += 1


def _version_key(conv, bn):
    key = [conv.weight._version, conv.weight.data_ptr()]
    trainable = conv.weight.requires_grad or (
        bn is not None and bn.weight is not None and bn.weight.requires_grad)
    if trainable:
        key.append(("gen", _GEN[0]))
    if conv.bias is not None:
        key += [conv.bias._version]
    if bn is not None:
        for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var):
            if t is not None:
                key += [t._version, t.data_ptr()]
    return tuple(key)


@torch.no_grad()
def _packed(conv, bn):
    key = _version_key(conv, bn)
    cache = getattr(conv, "_mda_pack", None)
    if cache is not None and cache[0] == key and cache[1] is bn:
        return cache[2], cache[3]
    w = conv.weight.detach().float()
    cout = w.shape[0]
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(cout, device=w.device)
    if bn is not None:
        g = bn.weight.detach().float() if bn.weight is not None else torch.ones(cout, device=w.device)
        beta = bn.bias.detach().float() if bn.bias is not None else torch.zeros(cout, device=w.device)
        s = g / torch.sqrt(bn.running_var.float() + bn.eps)
        w = w * s.reshape(-1, 1, 1, 1)
        b = beta + (b - bn.running_mean.float()) * s
    from .hip_train import needs_channel_pad
    if needs_channel_pad(w.shape[1]):  # stem: input padded to 8 channels
        w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 8 - w.shape[1]))
    K = w.shape[1] * w.shape[2] * w.shape[3]
    Kp = (K + 63) // 64 * 64
    wp = torch.zeros(cout, Kp, dtype=torch.bfloat16, device=w.device)
    wp[:, :K] = w.permute(0, 2, 3, 1).reshape(cout, K).to(torch.bfloat16)
    b = b.contiguous()
    conv._mda_pack = (key, bn, wp, b)
    return wp, b


def _nhwc_bf16(t):
    if t.dtype != torch.bfloat16:
        t = t.to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


@torch.no_grad()
def _dw_packed(conv, bn):
    """Depthwise: BN folded into fp32 tap-major [9, C] weights + bias (cached)."""
    key = _version_key(conv, bn)
    cache = getattr(conv, "_mda_dwpack", None)
    if cache is not None and cache[0] == key and cache[1] is bn:
        return cache[2], cache[3]
    from .hip_train import dw_pack
    C = conv.out_channels
    dev = conv.weight.device
    b = conv.bias.detach().float() if conv.bias is not None else torch.zeros(C, device=dev)
    s = None
    if bn is not None:
        g = bn.weight.detach().float() if bn.weight is not None else torch.ones(C, device=dev)
        beta = bn.bias.detach().float() if bn.bias is not None else torch.zeros(C, device=dev)
        s = (g / torch.sqrt(bn.running_var.float() + bn.eps)).contiguous()
        b = beta + (b - bn.running_mean.float()) * s
    wp = dw_pack(conv.weight, s)
    b = b.contiguous()
    conv._mda_dwpack = (key, bn, wp, b)
    return wp, b


def _dw_conv_bn_act(x, conv, bn, act, residual, want_preact):
    wp, bias = _dw_packed(conv, bn)
    x = _nhwc_bf16(x)
    N, C, H, W = x.shape
    s, p = conv.stride[0], conv.padding[0]
    Ho = (H + 2 * p - 3) // s + 1
    Wo = (W + 2 * p - 3) // s + 1
    y = torch.empty((N, C, Ho, Wo), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    pre = torch.empty_like(y) if want_preact else None
    res = _nhwc_bf16(residual) if residual is not None else None
    _ext.call("mda_dw_fwd", x, wp, None, bias, res, y, pre, N, H, W, C, Ho, Wo, 3, 3, s, p,
              _ACT[act])
    return y, pre


def conv_bn_act(x, conv, bn, act, residual, want_preact):
    if conv.groups != 1:
        return _dw_conv_bn_act(x, conv, bn, act, residual, want_preact)
    wp, bias = _packed(conv, bn)
    from .hip_train import needs_channel_pad, pad_channels8
    x = pad_channels8(x) if needs_channel_pad(x.shape[1]) else _nhwc_bf16(x)
    N, Cin, H, W = x.shape
    Cout = conv.out_channels
    KH, KW = conv.kernel_size
    s, p = conv.stride[0], conv.padding[0]
    Ho = (H + 2 * p - KH) // s + 1
    Wo = (W + 2 * p - KW) // s + 1
    y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    pre = torch.empty_like(y) if want_preact else None
    res = _nhwc_bf16(residual) if residual is not None else None
    M = N * Ho * Wo
    tile, splits = conv_plan(M, Cout, wp.shape[1])
    part = torch.empty(splits * M * Cout, dtype=torch.float32, device=x.device) if splits > 1 else None
    _ext.call("mda_conv_fwd", x, wp, None, bias, res, y, pre, part, N, H, W, Cin, Ho, Wo, Cout,
              KH, KW, s, p, wp.shape[1], _ACT[act], tile, splits)
    return y, pre


_PLANS: dict = {}


def conv_plan(M, Cout, Kp):
    key = (M, Cout, Kp)
    plan = _PLANS.get(key)
    if plan is None:
        import ctypes
        t, s = ctypes.c_int64(0), ctypes.c_int64(0)
        _ext.call("mda_conv_plan", M, Cout, Kp, t, s)
        plan = _PLANS[key] = (t.value, s.value)
    return plan
