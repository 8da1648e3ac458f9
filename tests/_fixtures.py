"""Stored reference outputs (``tests/fixtures/*.safetensors``) for the parity
tests.  They were produced once by ``scripts/gen_ref_fixtures.py`` from the
reference's own sources; tests only read tensors here, nothing of the
reference is imported or executed in a test process."""
import functools
import os

from safetensors.torch import load_file

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")


@functools.lru_cache(maxsize=None)
def load(name: str) -> dict:
    return load_file(os.path.join(DIR, name + ".safetensors"))


def case(name: str, key: str):
    """All tensors of one case, ``{"in0": ..., "loss": ..., "grad0": ...}``."""
    d = load(name)
    p = key + "/"
    return {k[len(p):]: v.clone() for k, v in d.items() if k.startswith(p)}
