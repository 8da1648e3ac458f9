"""Load individual reference source files (read-only) for numerical parity tests.

Only pure-PyTorch modules are loaded (distiller loss functions, the DOT
optimizer); relative imports are satisfied by a synthetic package.  Tests
that use this skip when the reference tree is not mounted.
"""
import importlib.util
import os
import sys
import types

REF = os.environ.get("MDA_REFERENCE", "/root/reference")
DIST = os.path.join(REF, "mdistiller", "distillers")
ENGINE = os.path.join(REF, "mdistiller", "engine")


def available() -> bool:
    return os.path.isdir(DIST)


def _pkg(name, path):
    if name in sys.modules:
        return sys.modules[name]
    pkg = types.ModuleType(name)
    pkg.__path__ = [path]
    sys.modules[name] = pkg
    return pkg


def load(kind: str, mod: str):
    """``load("distillers", "KD")`` -> the reference module object."""
    base = DIST if kind == "distillers" else ENGINE
    pkg_name = f"_mdaref_{kind}"
    _pkg(pkg_name, base)
    full = f"{pkg_name}.{mod}"
    if full in sys.modules:
        return sys.modules[full]
    spec = importlib.util.spec_from_file_location(full, os.path.join(base, mod + ".py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules[full] = m
    spec.loader.exec_module(m)
    return m
