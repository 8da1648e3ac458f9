"""Distiller registry (reference `mdistiller/distillers/__init__.py:16-31`).

Keys are the ``DISTILLER.TYPE`` strings of the shipped YAMLs.
"""
from ._base import Distiller, Vanilla
from .KD import KD
from .DKD import DKD

distiller_dict = {
    "NONE": Vanilla,
    "KD": KD,
    "DKD": DKD,
}

try:  # feature-based methods (registered as they are added)
    from .AT import AT
    from .FitNet import FitNet
    from .NST import NST
    from .PKT import PKT
    from .SP import SP
    from .RKD import RKD
    from .KDSVD import KDSVD
    from .VID import VID
    from .OFD import OFD
    from .CRD import CRD
    from .ReviewKD import ReviewKD
    distiller_dict.update({"AT": AT, "FITNET": FitNet, "NST": NST, "PKT": PKT, "SP": SP,
                           "RKD": RKD, "KDSVD": KDSVD, "VID": VID, "OFD": OFD, "CRD": CRD,
                           "REVIEWKD": ReviewKD})
except ImportError:  # pragma: no cover
    pass
