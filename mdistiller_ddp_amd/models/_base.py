"""Model contract shared by the whole zoo.

Every model returns ``(logits, feats)`` where ``feats`` is a dict with

* ``"feats"``        -- ``[stem, stage_1, ..., stage_N]`` activated features,
* ``"preact_feats"`` -- the same positions before the final activation,
* ``"pooled_feat"``  -- the globally pooled vector fed to the classifier.

The list is *stem-inclusive* (the upstream mdistiller contract).  The
reference fork dropped the stem entry in its models but not in its distillers
(SURVEY D6), which breaks OFD/ReviewKD and silently drops a stage in
AT/NST/KDSVD/VID; keeping the stem at index 0 makes every ``[1:]`` slice in
the distillers select exactly the N stages again.

``ModelBase`` is the staged-forward API of `mdistiller/models/_base.py:16-40`
(``forward_stem -> get_layers -> forward_pool -> get_head``), implemented by
every model here (the reference leaves ``get_arch`` abstract in four families,
SURVEY D1, and its ``get_layers`` references an undefined ``x``, D7).
"""
from __future__ import annotations

from typing import Literal

import torch
from torch import nn


class Lambda(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, *args, **kwargs):
        return self.fn(*args, **kwargs)


class ModelBase:
    """Mixin: staged forward + feature-request plumbing."""

    arch: str = "cnn"
    # Which intermediate outputs the consumer needs.  "preact" additionally asks
    # the fused HIP kernels to store pre-activation tensors.
    _need_preact: bool = True

    def get_arch(self) -> Literal["cnn", "transformer"]:
        return self.arch

    def activate(self, x: torch.Tensor) -> torch.Tensor:
        return nn.functional.relu(x)

    def request_features(self, preact: bool = True) -> None:
        """Tell the model whether pre-activation features are consumed."""
        for m in self.modules():
            if isinstance(m, ModelBase) or hasattr(m, "_need_preact"):
                m._need_preact = preact

    # staged API ----------------------------------------------------------------
    def forward_stem(self, x):  # pragma: no cover - overridden
        raise NotImplementedError

    def get_layers(self) -> nn.Sequential:  # pragma: no cover - overridden
        raise NotImplementedError

    def forward_pool(self, x):  # pragma: no cover - overridden
        raise NotImplementedError

    def get_head(self) -> nn.Module:  # pragma: no cover - overridden
        raise NotImplementedError

    def get_stage_channels(self):
        return list(self.stage_channels)


class PreactStage(nn.Module):
    """Adapter for ``get_layers()``: activated input -> stage pre-activation.

    Wraps a stage whose forward returns ``(out, preact)`` so the staged API
    (`_base.py:42-74` ``test_model``) sees one tensor in, one tensor out.
    """

    def __init__(self, stage: nn.Module):
        super().__init__()
        self.stage = stage

    def forward(self, x):
        self.stage._need_preact = True
        for m in self.stage.modules():
            if hasattr(m, "_need_preact"):
                m._need_preact = True
        out = self.stage(x)
        return out[1] if isinstance(out, tuple) else out


def run_staged(model: ModelBase, x: torch.Tensor):
    """Run the staged forward; returns (logits, preact_feats, feats, pooled)."""
    y = model.forward_stem(x)
    preacts = []
    for layer in model.get_layers():
        y = layer(model.activate(y))
        preacts.append(y)
    feats = [model.activate(p) for p in preacts]
    pooled = model.forward_pool(y)
    logits = model.get_head()(pooled)
    return logits, preacts, feats, pooled


def check_staged_forward(model: ModelBase, x: torch.Tensor, atol=1e-5, rtol=1e-4) -> dict:
    """Staged forward == forward, stage by stage (stem entry excluded).

    Returns a dict of booleans (the reference's ``test_model`` result shape).
    """
    was_training = model.training
    model.eval()
    with torch.no_grad():
        logits, f = model(x)
        l2, pre2, feats2, pooled2 = run_staged(model, x)
    model.train(was_training)

    def close(a, b):
        return a.shape == b.shape and torch.allclose(a.float(), b.float(), atol=atol, rtol=rtol)

    res = {
        "logits": close(logits, l2),
        "preact_feats": [close(a, b) for a, b in zip(f["preact_feats"][1:], pre2)],
        "feats": [close(a, b) for a, b in zip(f["feats"][1:], feats2)],
        "pooled_feat": close(f["pooled_feat"].reshape(pooled2.shape), pooled2),
        "num_stages_match": len(f["feats"]) - 1 == len(feats2),
    }
    res["all"] = all([res["logits"], res["pooled_feat"], res["num_stages_match"],
                      *res["preact_feats"], *res["feats"]])
    return res
