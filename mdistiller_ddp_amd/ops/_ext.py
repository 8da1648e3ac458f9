"""ctypes bindings for the native libraries built by :mod:`.build`.

Every device launcher exported by ``libmda_hip.so`` has a plain C ABI:
``int mda_<name>(<pointers/ints/floats>..., hipStream_t stream)`` returning a
``hipError_t``.  Signatures are declared once in :data:`SIGNATURES` with a
compact code per argument:

``p`` device/host pointer (a ``torch.Tensor`` is converted via ``data_ptr()``),
``i`` int64, ``f`` float32, ``s`` stream (defaults to the current torch stream).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from . import build as _build

_lock = threading.Lock()
_LIBS: dict = {}
_FAILED: dict = {}
LOADED_PATHS: list = []

_CT = {"p": ctypes.c_void_p, "i": ctypes.c_int64, "f": ctypes.c_float, "s": ctypes.c_void_p,
       "d": ctypes.c_double}

# name -> argument codes (stream last).  Kept in sync with csrc/*.hip `extern "C"` launchers.
SIGNATURES = {
    # losses (csrc/losses.hip)
    "mda_logit_loss": "iiippppppppiifffffpfps",
    "mda_axpby": "ipppppis",
    # feature losses (csrc/feat.hip)
    "mda_at_loss": "iipppppp" + "iiii" + "fs",
    # relational losses on the batch Gram (csrc/relation.hip)
    "mda_gram_plan": "ipp",
    "mda_gram_partial": "ppp" + "i" * 7 + "s",
    "mda_relation_core": "piiiipps",
    "mda_rkd_loss": "piiii" + "fff" + "pppppps",
    "mda_gram_bwd": "ppppiis",
    # graph-external events (csrc/events.hip)
    "mda_event_create": "p",
    "mda_event_destroy": "p",
    "mda_event_record": "pis",
    "mda_clock_probe": "pis",
    "mda_stream_wait_event": "pis",
    # convolution (csrc/conv_igemm.hip)
    "mda_conv_fwd": "pppppppp" + "i" * 15 + "s",
    "mda_conv_plan": "iiipp",
    "mda_conv_set_stamps": "p",
    "mda_conv_fwd_bnstats": "ppppp" + "i" * 15 + "p" * 8 + "ff" + "ps",
    "mda_conv_dgrad": "pppp" + "i" * 14 + "s",
    "mda_conv_dgrad_res": "ppppp" + "i" * 14 + "s",
    "mda_conv_dgrad_bnsum": "ppppp" + "i" * 14 + "ppp" + "i" + "p" + "s",
    "mda_conv_dgrad_bnsum_g": "ppppp" + "i" * 14 + "ppp" + "i" + "p" + "i" + "p" + "ii" + "s",
    "mda_conv_fwd_bnacc_g": "ppppp" + "i" * 14 + "i" + "s",
    "mda_pack_conv_weights_gc": "ppp" + "i" * 7 + "s",
    "mda_channel_gather": "ppp" + "iii" + "s",
    "mda_gather2": "pppp" + "i" + "ppi" + "iii" + "s",
    "mda_act_bwd": "pppp" + "ii" + "s",
    "mda_vid_loss": "ppp" + "ii" + "f" + "pp" + "s",
    "mda_vid_bwd": "pppp" + "p" + "ii" + "f" + "pp" + "s",
    "mda_nst_fwd": "p" + "ii" + "p" + "s",
    "mda_dw_fwd_bnacc": "pppp" + "i" * 10 + "s",
    "mda_nst_bwd": "p" + "ii" + "pp" + "s",
    "mda_conv_wgrad": "pppp" + "i" * 13 + "fiii" + "ii" + "s",
    "mda_conv_wgrad_nored": "pppp" + "i" * 13 + "fiii" + "i" + "s",
    "mda_conv1x1_bnacc_apply": "pppp" + "i" * 9 + "pp" + "ii" + "ppppp" + "ff" + "p" + "ppp" + "i" + "s",
    "mda_conv_wgrad_nored_bn": "pppp" + "i" * 15 + "pppp" + "iii" + "pppppp" + "pppp" + "s",
    "mda_wgrad_reduce_multi": "pis",
    "mda_pack_conv_weights_grouped": "ppp" + "i" * 7 + "s",
    "mda_pad_channels": "ippiiis",
    # max pooling (csrc/pool.hip)
    "mda_maxpool_fwd": "ppp" + "i" * 9 + "s",
    "mda_maxpool_bwd": "ppp" + "i" * 9 + "s",
    "mda_shuffle_tail_fwd": "pppp" + "i" * 7 + "s",
    "mda_shuffle_tail_bwd": "ppppp" + "i" * 7 + "s",
    "mda_pack_conv_weights_pad": "pp" + "i" * 6 + "s",
    "mda_wgrad_plan": "iiiiiiiiiip",
    "mda_conv_dgrad_bnsum2": "pppiiiiiiiiiiiipppippppiis",
    "mda_pack_conv_weights": "ppp" + "i" * 6 + "s",
    "mda_pack_conv_weights_multi": "piiis",
    "mda_pack_tiles": "iiiip",
    # depthwise 3x3 conv (csrc/dwconv.hip)
    "mda_dw_pack": "pppiis",
    "mda_dw_fwd": "ppppppp" + "i" * 11 + "s",
    "mda_dw_dgrad": "ppp" + "i" * 10 + "s",
    "mda_dw_wgrad_blocks": "iiiip",
    "mda_dw_wgrad": "pppp" + "i" * 12 + "s",
    "mda_dw_wgrad_blocks2": "i" * 8 + "p",
    # training-mode BatchNorm (csrc/bn.hip)
    "mda_bn_stats": "pii" + "pp" + "pppp" + "pppp" + "ffps",
    "mda_bn_apply": "pppppp" + "iii" + "s",
    "mda_bn_bwd_reduce": "pppppppp" + "iii" + "ppppp" + "s",
    "mda_bn_bwd_apply": "p" * 11 + "iii" + "s",
    "mda_bn_tune": "ii",
    "mda_bn_stats2": "piip" + "pppp" + "pppp" + "ffps",
    "mda_bn_bwd_reduce2": "pppppppp" + "iii" + "pppp" + "s",
    "mda_bn_finalize": "piii" + "pppppppp" + "ffps",
    # fused BN through a per-stream slot (csrc/bn.hip, csrc/bnslot.h)
    "mda_bn_region_bytes": "ip",
    "mda_bn_stats_acc": "piips",
    "mda_bn_apply_fin": "ppii" + "ppppp" + "ff" + "p" + "ppp" + "i" + "s",
    "mda_bn_apply_fin_vr": "ppii" + "ppppp" + "ff" + "p" + "ppp" + "i" + "pppppp" + "ff" + "p" + "s",
    "mda_bn_bwd_fused": "ppppp" + "p" + "iii" + "pp" + "pp" + "ppp" + "ppp" + "p" + "iiii" + "s",
    "mda_bn_bwd_apply_reg": "pppp" + "p" + "iii" + "p" + "pp" + "ppp" + "ppp" + "p" + "iiii" + "s",
    "mda_conv_fwd_bnacc": "ppppp" + "i" * 14 + "s",
    # CRD memory (csrc/crd.hip)
    "mda_crd_scores": "ppppiiifs",
    "mda_crd_grad": "ppppppiiifs",
    "mda_crd_update": "pppiifs",
    "mda_embed_fwd": "ppppp" + "iii" + "s",
    "mda_embed_bwd": "ppppp" + "pppp" + "iii" + "s",
    # classifier head + metrics (csrc/head.hip)
    "mda_pool_fc_fwd": "ipppppiiiis",
    "mda_pool_fc_bwd": "ippppppp" + "iiiii" + "s",
    "mda_sym_eig": "piiipp" + "s",
    # KDSVD alignment + RBF + L2 after the eigensolver (csrc/kdsvd.hip)
    "mda_kdsvd_post": "ppppp" + "iii" + "pp" + "pp" + "s",
    "mda_kdsvd_gram": "pii" + "s",
    "mda_kdsvd_gram_apply": "pi" + "s",
    "mda_sym_eig_multi": "pii" + "s",
    "mda_pool_fc_bwd_bn": "ippppppp" + "iiiii" + "pppip" + "p" + "s",
    "mda_meters_update": "ippii" + "pppp" + "ips",
    # ReviewKD HCL + ABF (csrc/reviewkd.hip)
    "mda_hcl_loss": "piiipfpfps",
    "mda_attn_fwd": "pppiiifs",
    "mda_channel_shuffle": "ppiiis",
    "mda_ofd_loss": "ppppppp" + "ii" + "fs",
    "mda_attn_bwd": "ppppppiiifs",
    "mda_abf_fwd": "pppppp" + "iiiiii" + "s",
    "mda_abf_bwd_blocks": "iiiip",
    "mda_abf_bwd": "ppppppppppp" + "iiiiii" + "ii" + "s",
    # detection: multi-level ROIAlign + NMS (csrc/det.hip)
    "mda_roi_align_fwd": "ii" + "pppppp" + "iiiiii" + "s",
    "mda_roi_align_bwd": "ii" + "pppppp" + "iiiiii" + "s",
    "mda_nms": "pifpipps",
    "mda_deform_im2col": "i" + "pppp" + "p" + "s",
    "mda_deform_col2im": "i" + "pppp" + "ppp" + "p" + "s",
    # data augmentation (csrc/aug.hip)
    "mda_crop_flip_norm": "ppppppp" + "iiiiii" + "s",
    # optimizers (csrc/optim.hip)
    "mda_sgd_step": "ppppfffpfis",
    "mda_dot_step": "pppppppffffiis",
    "mda_adam_step": "ppppppffffifpfis",
    "mda_sq_norm": "pipppfs",
    "mda_scale_inplace": "ppis",
    "mda_multi_copy": "pis",
}

HOST_SIGNATURES = {
    "mdah_crd_sample": "ppppppiiiii",
    "mdah_alias_build": "pppi",
}


def gpu_box() -> bool:
    """A GPU is present (without initialising HIP)."""
    try:
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def _declare(lib, table):
    for name, codes in table.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = [_CT[c] for c in codes]
        fn.restype = ctypes.c_int


def load(required: bool = False, kind: str = "hip"):
    """Load (building first if stale) a native library; returns the ctypes handle or None."""
    with _lock:
        if kind in _LIBS:
            return _LIBS[kind]
        if kind in _FAILED and not required:
            return None
        try:
            if os.environ.get("MDA_NO_BUILD", "0") != "1":
                _build.build(kind)
            path = _build.HIP_LIB if kind == "hip" else _build.HOST_LIB
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            _declare(lib, SIGNATURES if kind == "hip" else HOST_SIGNATURES)
            _LIBS[kind] = lib
            LOADED_PATHS.append(path)
            return lib
        except Exception as e:  # pragma: no cover - exercised on broken toolchains
            _FAILED[kind] = e
            if required:
                raise RuntimeError(f"native library '{kind}' unavailable: {e}") from e
            return None


def available(kind: str = "hip") -> bool:
    return load(required=False, kind=kind) is not None


def _arg(a, code):
    if code in ("p", "s"):
        if a is None:
            return None
        if isinstance(a, torch.Tensor):
            return a.data_ptr()
        if isinstance(a, ctypes._SimpleCData):
            return ctypes.addressof(a)
        return int(a)
    if code == "i":
        return int(a)
    return float(a)


NOT_SERVED = -1  # csrc/common.h MDA_NOT_SERVED: an optional fused launcher did not launch


def call(name: str, *args, stream=None, ok=(0,)):
    """Invoke a HIP launcher; ``stream`` defaults to the current torch stream.
    Returns the launcher's status; any status outside ``ok`` raises."""
    lib = load(required=True)
    fn = getattr(lib, name)
    codes = SIGNATURES[name]
    has_stream = codes.endswith("s")
    nargs = len(codes) - (1 if has_stream else 0)
    if len(args) != nargs:
        raise TypeError(f"{name}: expected {nargs} args, got {len(args)}")
    conv = [_arg(a, c) for a, c in zip(args, codes[:nargs])]
    if has_stream:
        if stream is None:
            stream = torch.cuda.current_stream().cuda_stream
        conv.append(stream)
    err = fn(*conv)
    if err not in ok:
        raise RuntimeError(f"{name} failed with hipError {err}")
    return err


def host_call(name: str, *args):
    lib = load(required=True, kind="host")
    fn = getattr(lib, name)
    codes = HOST_SIGNATURES[name]
    conv = [_arg(a, c) for a, c in zip(args, codes)]
    return fn(*conv)
