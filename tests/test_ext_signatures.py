"""The ctypes signature table must match every ``MDA_API`` launcher in csrc."""
import os
import re

from mdistiller_ddp_amd.ops import _ext

CSRC = os.path.join(os.path.dirname(_ext.__file__), "csrc")

_CODE = [
    (re.compile(r"hipStream_t"), "s"),
    (re.compile(r"\*"), "p"),
    (re.compile(r"\b(float)\b"), "f"),
    (re.compile(r"\b(double)\b"), "d"),
    (re.compile(r"\b(int64_t|int|unsigned|uint32_t|long)\b"), "i"),
]


def _code(arg):
    for rx, c in _CODE:
        if rx.search(arg):
            return c
    raise AssertionError(f"unknown arg type: {arg}")


def _declared(ext, api):
    out = {}
    root = CSRC if ext == ".hip" else os.path.join(CSRC, "host")
    for f in os.listdir(root):
        if not f.endswith(ext):
            continue
        src = open(os.path.join(root, f)).read()
        for m in re.finditer(api + r"\s+\w+\s+(\w+)\s*\(([^)]*)\)", src):
            args = [a.strip() for a in m.group(2).split(",") if a.strip()]
            out[m.group(1)] = "".join(_code(a) for a in args)
    return out


def test_hip_signatures_match_sources():
    decl = _declared(".hip", "MDA_API")
    assert decl, "no launchers found"
    for name, codes in decl.items():
        assert name in _ext.SIGNATURES, f"{name} missing from SIGNATURES"
        assert _ext.SIGNATURES[name] == codes, (name, _ext.SIGNATURES[name], codes)
    for name in _ext.SIGNATURES:
        assert name in decl, f"{name} in SIGNATURES but not in csrc"


def test_host_signatures_match_sources():
    decl = _declared(".cpp", "MDA_HOST_API")
    for name, codes in decl.items():
        assert name in _ext.HOST_SIGNATURES, name
        assert _ext.HOST_SIGNATURES[name] == codes, (name, _ext.HOST_SIGNATURES[name], codes)
