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


MODELS = os.path.join(REF, "mdistiller", "models")


def load_model_module(sub: str, mod: str):
    """``load_model_module("cifar", "ShuffleNetv1")`` -> the reference model
    module (its ``from .._base import ...`` resolves to the reference's
    models/_base.py through synthetic packages)."""
    root = "_mdaref_models"
    _pkg(root, MODELS)
    base_full = f"{root}._base"
    if base_full not in sys.modules:
        spec = importlib.util.spec_from_file_location(base_full, os.path.join(MODELS, "_base.py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[base_full] = m
        spec.loader.exec_module(m)
    _pkg(f"{root}.{sub}", os.path.join(MODELS, sub))
    full = f"{root}.{sub}.{mod}"
    if full in sys.modules:
        return sys.modules[full]
    spec = importlib.util.spec_from_file_location(full, os.path.join(MODELS, sub, mod + ".py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules[full] = m
    spec.loader.exec_module(m)
    return m
