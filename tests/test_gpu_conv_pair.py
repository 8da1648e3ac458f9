"""A residual block's conv1 and projection shortcut share their input: the
shortcut's input gradient is folded into conv1's strided dgrad launch
(csrc/conv_igemm.hip ``mda_conv_dgrad_bnsum2``), checked against the two
separate dgrads."""
import copy

import pytest
import torch

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.ops import hip_train

pytestmark = pytest.mark.gpu


def _cfg(student):
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    return cfg


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("student", ["resnet8x4", "resnet32x4"])
def test_folded_shortcut_dgrad_matches_separate(student):
    """The projection shortcut's input gradient folded into conv1's strided
    dgrad (one launch, no parked gradient / residual add) == the two dgrads:
    the first step's gradients, and the parameters after a few steps at a
    small learning rate (a random teacher's KD at the default rate amplifies
    the different bf16 rounding of the two orders of summation)."""
    cfg = _cfg(student)
    cfg.SOLVER.LR = 0.005
    torch.manual_seed(1)
    d1 = build_distiller(cfg, 100, "cuda")
    d2 = copy.deepcopy(d1)
    ld = SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=1, channels_last=True)
    batches = [next(iter(ld)) for _ in range(3)]
    out = []
    for d, merge in ((d1, True), (d2, False)):
        hip_train.set_dgrad_merge(merge)
        try:
            d.train()
            st = TrainStep(d, cfg, "cuda", use_graph=False, dtype=torch.bfloat16)
            st.set_epoch(1.0)
            n0 = hip_train._MERGE_COUNT[0]
            g0 = None
            for b in batches:
                st.step({k: v.clone() for k, v in b.items()})
                if g0 is None:
                    torch.cuda.synchronize()
                    g0 = st.flat.grads.clone()
            torch.cuda.synchronize()
            merged = hip_train._MERGE_COUNT[0] - n0
        finally:
            hip_train.set_dgrad_merge(True)
        out.append((st.flat.data.clone(), g0, merged))
    (p1, g1, n1), (p2, g2, n2) = out
    # two stride-2 downsampling blocks fold per step (the stride-1 one does not)
    assert n1 == 2 * len(batches) and n2 == 0, (n1, n2)
    assert _rel(g1, g2) < 1e-2, _rel(g1, g2)
    assert _rel(p1, p2) < 1e-3, _rel(p1, p2)


@pytest.mark.parametrize("shape", [(16, 64, 32, 128), (64, 128, 16, 256), (64, 64, 16, 64)])
def test_dgrad_bnsum2_kernel(shape):
    """mda_conv_dgrad_bnsum2 alone: dgrad of a 3x3/s2/p1 conv + dgrad of a
    1x1/s2 conv on the same input, in one launch, vs the two separate MFMA
    dgrads summed in fp32."""
    from mdistiller_ddp_amd.ops import _ext
    N, Cin, H, Cout = shape
    torch.manual_seed(3)
    Ho = H // 2
    w1 = (torch.randn(Cout, Cin, 3, 3, device="cuda") * 0.1).to(torch.bfloat16).float()
    w2 = (torch.randn(Cout, Cin, 1, 1, device="cuda") * 0.1).to(torch.bfloat16).float()
    dy1 = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy2 = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    _, wt1, _, KpT1 = hip_train.pack_weights(w1, True)
    _, wt2, _, KpT2 = hip_train.pack_weights(w2, True)
    dx = torch.empty(N, Cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    rc = _ext.call("mda_conv_dgrad_bnsum2", dy1, wt1, dx, N, H, H, Cin, Ho, Ho, Cout, 3, 3, 2, 1,
                   KpT1, None, None, None, 0, None, None, dy2, wt2, Cout, KpT2, ok=(0, _ext.NOT_SERVED))
    assert rc == 0
    a = hip_train.conv_dgrad(dy1, w1, (N, Cin, H, H), 2, 1).float()
    b = hip_train.conv_dgrad(dy2, w2, (N, Cin, H, H), 2, 0).float()
    ref = a + b
    rel = ((dx.float() - ref).norm() / ref.norm()).item()
    assert rel < 1e-2, rel
