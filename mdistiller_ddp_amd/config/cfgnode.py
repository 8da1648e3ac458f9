"""A small yacs-compatible hierarchical config node.

The reference builds its whole config surface on ``yacs.config.CfgNode``
(`mdistiller/engine/cfg.py:1,26`).  yacs is not part of this image, and the
framework must keep the shipped YAMLs and the ``KEY VALUE`` CLI overrides
byte-compatible, so this module re-implements the subset of the yacs contract
the reference relies on:

* attribute access on a ``dict`` subclass (``cfg.SOLVER.LR``);
* ``merge_from_file`` / ``merge_from_other_cfg`` / ``merge_from_list`` with
  unknown-key rejection and type coercion (yacs semantics: a value merged
  into an existing key must keep that key's type, with the usual
  str/tuple/list/int->float allowances);
* ``freeze`` / ``defrost`` / ``is_frozen`` (immutability is recursive);
* ``clone`` and ``dump`` (YAML text, round-trips through ``load_cfg``).
"""
from __future__ import annotations

import ast
import copy
import io
from typing import Any, Iterable

import yaml

_VALID_TYPES = (tuple, list, str, int, float, bool, type(None))


class CfgNode(dict):
    IMMUTABLE = "__immutable__"
    NEW_ALLOWED = "__new_allowed__"

    def __init__(self, init_dict: dict | None = None, key_list: list | None = None,
                 new_allowed: bool = False):
        init_dict = {} if init_dict is None else init_dict
        key_list = [] if key_list is None else key_list
        for k, v in list(init_dict.items()):
            if isinstance(v, dict) and not isinstance(v, CfgNode):
                init_dict[k] = CfgNode(v, key_list + [k], new_allowed=new_allowed)
        super().__init__(init_dict)
        self.__dict__[CfgNode.IMMUTABLE] = False
        self.__dict__[CfgNode.NEW_ALLOWED] = new_allowed

    # ------------------------------------------------------------------ access
    def __getattr__(self, name: str) -> Any:
        if name in self:
            return self[name]
        raise AttributeError(name)

    def __setattr__(self, name: str, value: Any) -> None:
        if self.is_frozen():
            raise AttributeError(
                f"Attempted to set {name} to {value}, but CfgNode is immutable")
        if name in self.__dict__:
            raise AttributeError(f"Invalid attempt to modify internal CfgNode state: {name}")
        if isinstance(value, dict) and not isinstance(value, CfgNode):
            value = CfgNode(value)
        self[name] = value

    def __setitem__(self, key, value):
        if self.__dict__.get(CfgNode.IMMUTABLE, False):
            raise AttributeError(f"Attempted to set {key}, but CfgNode is immutable")
        super().__setitem__(key, value)

    def __deepcopy__(self, memo):
        out = CfgNode(new_allowed=self.__dict__[CfgNode.NEW_ALLOWED])
        for k, v in self.items():
            dict.__setitem__(out, k, copy.deepcopy(v, memo))
        return out

    def __reduce__(self):
        return (_rebuild, (self.to_dict(),))

    def __str__(self) -> str:
        return self.dump()

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}({dict.__repr__(self)})"

    # --------------------------------------------------------------- freezing
    def freeze(self) -> None:
        self._set_immutable(True)

    def defrost(self) -> None:
        self._set_immutable(False)

    def is_frozen(self) -> bool:
        return self.__dict__[CfgNode.IMMUTABLE]

    def _set_immutable(self, flag: bool) -> None:
        self.__dict__[CfgNode.IMMUTABLE] = flag
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_immutable(flag)

    # ---------------------------------------------------------------- helpers
    def clone(self) -> "CfgNode":
        return copy.deepcopy(self)

    def to_dict(self) -> dict:
        return {k: (v.to_dict() if isinstance(v, CfgNode) else copy.deepcopy(v))
                for k, v in self.items()}

    def dump(self, **kwargs) -> str:
        return yaml.safe_dump(_to_plain(self), default_flow_style=False, **kwargs)

    def update(self, other=(), **kw):  # keep CfgNode children typed
        items = other.items() if isinstance(other, dict) else other
        for k, v in list(items) + list(kw.items()):
            if isinstance(v, dict) and not isinstance(v, CfgNode):
                v = CfgNode(v)
            self[k] = v

    # ---------------------------------------------------------------- merging
    def merge_from_file(self, cfg_filename: str) -> None:
        with open(cfg_filename, "r") as f:
            cfg = load_cfg(f)
        self.merge_from_other_cfg(cfg)

    def merge_from_other_cfg(self, cfg_other: "CfgNode") -> None:
        _merge_a_into_b(cfg_other, self, self, [])

    def merge_from_list(self, cfg_list: Iterable) -> None:
        cfg_list = list(cfg_list or [])
        if len(cfg_list) % 2 != 0:
            raise ValueError(f"Override list has odd length: {cfg_list}; it must be a list of pairs")
        root = self
        for full_key, v in zip(cfg_list[0::2], cfg_list[1::2]):
            key_list = full_key.split(".")
            d = self
            for subkey in key_list[:-1]:
                if subkey not in d:
                    raise KeyError(f"Non-existent key: {full_key}")
                d = d[subkey]
            subkey = key_list[-1]
            if subkey not in d:
                raise KeyError(f"Non-existent key: {full_key}")
            value = _decode_cfg_value(v)
            value = _check_and_coerce_cfg_value_type(value, d[subkey], subkey, full_key)
            d[subkey] = value
        del root

    def is_new_allowed(self) -> bool:
        return self.__dict__[CfgNode.NEW_ALLOWED]


def _rebuild(d: dict) -> CfgNode:
    return CfgNode(d)


def _to_plain(node):
    if isinstance(node, CfgNode):
        return {k: _to_plain(v) for k, v in node.items()}
    if isinstance(node, tuple):
        return [_to_plain(v) for v in node]
    if isinstance(node, list):
        return [_to_plain(v) for v in node]
    return node


def load_cfg(cfg_file_obj_or_str) -> CfgNode:
    """Load a config from a YAML string or file object (safe loader only)."""
    if isinstance(cfg_file_obj_or_str, str):
        data = yaml.safe_load(io.StringIO(cfg_file_obj_or_str))
    else:
        data = yaml.safe_load(cfg_file_obj_or_str)
    return CfgNode(data or {})


def _decode_cfg_value(value):
    if isinstance(value, dict):
        return CfgNode(value)
    if not isinstance(value, str):
        return value
    try:
        return ast.literal_eval(value)
    except (ValueError, SyntaxError):
        return value


def _check_and_coerce_cfg_value_type(replacement, original, key, full_key):
    original_type, replacement_type = type(original), type(replacement)
    if replacement_type == original_type:
        return replacement
    if original is None or replacement is None:
        return replacement
    casts = [(tuple, list), (list, tuple), (int, float)]
    for from_type, to_type in casts:
        if replacement_type == from_type and original_type == to_type:
            return to_type(replacement)
    if original_type is float and replacement_type is int:
        return float(replacement)
    if original_type is str and replacement_type is bool:
        # a mode key (``"auto"`` default) set from the command line as True / False
        return "true" if replacement else "false"
    raise ValueError(
        f"Type mismatch ({original_type} vs. {replacement_type}) with values "
        f"({original} vs. {replacement}) for config key: {full_key}")


def _merge_a_into_b(a: CfgNode, b: CfgNode, root: CfgNode, key_list: list) -> None:
    for k, v_ in a.items():
        full_key = ".".join(key_list + [k])
        v = copy.deepcopy(v_)
        v = _decode_cfg_value(v)
        if k in b:
            v = _check_and_coerce_cfg_value_type(v, b[k], k, full_key)
            if isinstance(v, CfgNode):
                if not isinstance(b[k], CfgNode):
                    raise ValueError(f"Cannot merge a node into a leaf at {full_key}")
                _merge_a_into_b(v, b[k], root, key_list + [k])
            else:
                b[k] = v
        elif b.is_new_allowed():
            b[k] = v
        else:
            raise KeyError(f"Non-existent config key: {full_key}")
