"""Training conv + BN finalize + apply in ONE launch (csrc/conv_igemm.hip
``mda_conv_fwd_bnfin``: grid barrier in the conv epilogue, ops/hip_train.py
``_FIN_ON``), and the BN backward finished inside the consumer's dgrad launch
(``mda_conv_dgrad_bnfin``, ``BnLink.can_finish``), against the separate
apply launches and against fp32 PyTorch."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.config import get_cfg
from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
from mdistiller_ddp_amd.engine.build import build_distiller
from mdistiller_ddp_amd.engine.step import TrainStep
from mdistiller_ddp_amd.ops import hip_train
from mdistiller_ddp_amd.ops.backend import use_backend



def _compiled():
    from mdistiller_ddp_amd.ops import _ext
    lib = _ext.load(required=False)
    return lib is not None and bool(lib.mda_bn_finish_compiled())


pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif("not _compiled()",
                                 reason="in-kernel BN finishes not compiled (MDA_BN_FINISH_KERNELS=0, "
                                        "the default: profiles/r5_ab.md)")]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,Cin,H,Cout,k,s,res,served", [(64, 64, 32, 64, 3, 1, False, True),
                                                         (64, 128, 16, 128, 3, 1, True, True),
                                                         (64, 128, 16, 256, 3, 2, False, True),
                                                         (64, 256, 8, 256, 3, 1, True, True),
                                                         # small M: a split-K plan, not served
                                                         (16, 64, 16, 64, 3, 1, False, False)])
def test_conv_bn_finish_layer_matches_fp32(N, Cin, H, Cout, k, s, res, served):
    """One conv + BN + ReLU (+ residual) layer: output, running statistics and
    the step count match the fp32 PyTorch layer; the finish kernel ran."""
    from mdistiller_ddp_amd.ops.nn import conv_bn_act
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, k // 2, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda()
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-0.2, 0.2)
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * (k // 2) - k) // s + 1
    r = (torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16)
         .contiguous(memory_format=torch.channels_last) if res else None)
    n0 = hip_train.bn_finish_count()
    with use_backend("hip"):
        y = conv_bn_act(x, conv, bn, "relu", residual=r)[0]
    torch.cuda.synchronize()
    assert hip_train.bn_finish_count() - n0 == int(served), "one-launch conv + BN path: unexpected"
    with torch.no_grad():
        z = bn_r(conv_r(x.float()))
        ref = F.relu(z + r.float() if res else z)
    assert _rel(y, ref) < 1e-2
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, bn_r.running_var, rtol=1e-3, atol=1e-4)
    assert int(bn.num_batches_tracked) == 1


def _cfg(student):
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    return cfg


@pytest.mark.parametrize("student,graph", [("resnet8x4", True), ("resnet20", False)])
def test_bn_finish_training_matches_two_launch_path(student, graph):
    """Whole training steps with the one-launch conv + BN path equal the
    two-launch path to within the BN-sum atomic-order spread, and the finish
    ran on most of the student's BN layers."""
    torch.manual_seed(0)
    d1 = build_distiller(_cfg(student), 100, "cuda")
    d2 = copy.deepcopy(d1)
    ld = SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=1, channels_last=True)
    batches = [next(iter(ld)) for _ in range(6)]
    out = []
    for d, fin in ((d1, True), (d2, False)):
        hip_train.set_bn_finish(fin)
        hip_train.set_bn_bwd_finish(fin)
        try:
            d.train()
            st = TrainStep(d, _cfg(student), "cuda", use_graph=graph, dtype=torch.bfloat16)
            st.set_epoch(1.0)
            n0 = hip_train.bn_finish_count()
            b0 = hip_train.bn_bwd_finish_count()
            losses = []
            for b in batches:
                _, l = st.step({k: v.clone() for k, v in b.items()})
                losses.append(float(sum(v for v in l.values())))
            torch.cuda.synchronize()
            n = (hip_train.bn_finish_count() - n0, hip_train.bn_bwd_finish_count() - b0)
        finally:
            hip_train.set_bn_finish(True)
            hip_train.set_bn_bwd_finish(True)
        out.append((st.flat.data.clone(), losses, n))
        assert hip_train.slot_errors() == 0
    (p1, l1, n1), (p2, l2, n2) = out
    assert n1[0] > 0 and n1[1] > 0 and n2 == (0, 0), (n1, n2)
    for a, b in zip(l1, l2):
        assert abs(a - b) <= 2e-2 * abs(b) + 1e-3, (l1, l2)
    assert _rel(p1, p2) < 5e-3


def _block_grads(stride, finish, seed=0):
    from mdistiller_ddp_amd.ops.nn import conv_bn_act
    torch.manual_seed(seed)
    C0, C1 = 64, 128
    c1 = nn.Conv2d(C0, C1, 3, stride, 1, bias=False).cuda()
    b1 = nn.BatchNorm2d(C1).cuda()
    c2 = nn.Conv2d(C1, C1, 3, 1, 1, bias=False).cuda()
    b2 = nn.BatchNorm2d(C1).cuda()
    for b in (b1, b2):
        b.weight.data.uniform_(0.5, 1.5)
        b.bias.data.uniform_(-0.2, 0.2)
    ref = [copy.deepcopy(m) for m in (c1, b1, c2, b2)]
    # conv2 runs on a 16x16 map: its dgrad grid (256 blocks) can be resident at once
    S = 16 * stride
    x = torch.randn(64, C0, S, S, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    params = [c1.weight, b1.weight, b1.bias, c2.weight]
    for q in params:
        q.grad = torch.zeros_like(q)  # bound gradients: dgamma / dbeta go straight in
    g = torch.randn(64, C1, 16, 16, device="cuda")
    hip_train.set_bn_bwd_finish(finish)
    try:
        n0 = hip_train.bn_bwd_finish_count()
        with use_backend("hip"):
            h = conv_bn_act(xa, c1, b1, "relu", private=True)[0]
            y = conv_bn_act(h, c2, b2, "relu")[0]
        (y.float() * g).sum().backward()
        torch.cuda.synchronize()
        n = hip_train.bn_bwd_finish_count() - n0
    finally:
        hip_train.set_bn_bwd_finish(True)
    got = [xa.grad] + [q.grad.clone() for q in params]
    xr = x.float().clone().requires_grad_(True)
    rc1, rb1, rc2, rb2 = ref
    yr = F.relu(rb2(rc2(F.relu(rb1(rc1(xr))))))
    (yr * g).sum().backward()
    want = [xr.grad, rc1.weight.grad, rb1.weight.grad, rb1.bias.grad, rc2.weight.grad]
    return got, want, n


@pytest.mark.parametrize("stride", [1, 2])
def test_bn_bwd_finish_block_matches_fp32(stride):
    """conv1 -> BN1 -> ReLU -> conv2 (h private): conv2's dgrad finishes BN1's
    backward.  The gradients of x, the conv weights and BN1's affine
    parameters equal the separate-apply path's to bf16 rounding, and both
    track fp32 autograd."""
    got, want, n = _block_grads(stride, True)
    base, _, n_off = _block_grads(stride, False)
    assert n == 1 and n_off == 0, "conv2's dgrad did not finish BN1's backward"
    assert hip_train.slot_errors() == 0
    for a, b in zip(got, base):
        assert _rel(a, b) < 1e-2, _rel(a, b)
    for a, b in zip(got, want):
        assert _rel(a, b) < 0.1, _rel(a, b)
    for a, b in zip(base, want):
        assert _rel(a, b) < 0.1, _rel(a, b)
