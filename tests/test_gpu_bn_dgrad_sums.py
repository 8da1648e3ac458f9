"""BN-backward sums in the consumer conv's dgrad epilogue (ops/hip_train.py
BnLink, conv_igemm.hip mda_conv_dgrad_bnsum, bn.hip mda_bn_bwd_apply_reg):
a training conv+BN+act layer whose output feeds the next native conv gets its
sum dz / sum dz*xhat from that conv's dgrad and runs one streaming backward
pass.  Checked against the same native layers with the link off (the
grid-barrier backward), against an fp32 PyTorch reference, under a residual
fork, and with an extra gradient on the linked activation (must fall back)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_train

pytestmark = pytest.mark.gpu

CHAINS = [
    # N, C0, C1, C2, H, stride of the consumer conv, consumer kernel
    (64, 64, 64, 64, 32, 1, 3),     # halo2 dgrad (Cin = 64)
    (64, 128, 128, 128, 16, 1, 3),  # halo dgrad
    (64, 256, 256, 256, 8, 1, 3),   # 8x8 maps
    (64, 64, 64, 128, 32, 2, 3),    # strided dgrad by parity class
    (64, 64, 64, 128, 32, 2, 1),    # 1x1 stride-2 projection
    (8, 24, 40, 48, 15, 1, 3),      # C / 8 not a power of two (VEC8 dgrad)
]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _chain(layers, x, g, extra=None):
    (c1, b1), (c2, b2) = layers
    xx = x.clone().requires_grad_(True)
    h, _ = hip_train.conv_bn_act_train(xx, c1, b1, "relu", None, False)
    out, _ = hip_train.conv_bn_act_train(h, c2, b2, "relu", None, False)
    loss = (out.float() * g).sum()
    if extra is not None:  # a second gradient on the linked activation
        loss = loss + (h.float() * extra).sum()
    loss.backward()
    return out, xx.grad


@pytest.mark.parametrize("shape", CHAINS)
def test_chain_matches_unlinked_and_fp32(shape):
    N, C0, C1, C2, H, s, k = shape
    torch.manual_seed(0)
    c1 = nn.Conv2d(C0, C1, 3, 1, 1, bias=False).cuda()
    b1 = nn.BatchNorm2d(C1).cuda()
    c2 = nn.Conv2d(C1, C2, k, s, k // 2, bias=False).cuda()
    b2 = nn.BatchNorm2d(C2).cuda()
    with torch.no_grad():
        for b in (b1, b2):
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.5, 0.5)
    mods = [(c1, b1), (c2, b2)]
    mods_off = copy.deepcopy(mods)
    mods_ref = copy.deepcopy(mods)
    x = torch.randn(N, C0, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * (k // 2) - k) // s + 1
    g = torch.randn(N, C2, Ho, Ho, device="cuda").to(torch.bfloat16).float()

    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = _chain(mods, x, g)
    hits, misses = hip_train.bn_dgrad_sums_count(reset=True)
    assert hits == 1 and misses == 0, (hits, misses)
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = _chain(mods_off, x, g)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    assert hip_train.bn_dgrad_sums_count(reset=True) == (0, 0)

    (r1, rb1), (r2, rb2) = mods_ref
    x2 = x.float().clone().requires_grad_(True)
    h = F.relu(rb1(r1(x2)))
    o = F.relu(rb2(r2(h)))
    o.backward(g)
    torch.cuda.synchronize()
    assert hip_train.slot_errors() == 0

    torch.testing.assert_close(out, out_off, atol=0, rtol=0)
    assert _rel(dx, dx_off) < 1e-2
    pairs = [(p.grad, q.grad) for m, mo in zip(mods, mods_off) for p, q in
             zip([m[0].weight, m[1].weight, m[1].bias], [mo[0].weight, mo[1].weight, mo[1].bias])]
    for a, b in pairs:
        assert _rel(a, b) < 1e-2
    assert _rel(dx, x2.grad) < 1e-1  # two bf16 conv+BN layers (both paths alike)
    refs = [r1.weight, rb1.weight, rb1.bias, r2.weight, rb2.weight, rb2.bias]
    mine = [c1.weight, b1.weight, b1.bias, c2.weight, b2.weight, b2.bias]
    for a, b in zip(mine, refs):
        assert _rel(a.grad, b.grad) < 1e-1


def test_extra_gradient_falls_back():
    """A feature loss on the linked activation adds a second gradient: autograd
    hands the BN a different tensor than the dgrad armed, so the layer must run
    the full backward on the summed gradient (and match the unlinked path)."""
    torch.manual_seed(1)
    c1 = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    b1 = nn.BatchNorm2d(64).cuda()
    c2 = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    b2 = nn.BatchNorm2d(64).cuda()
    mods = [(c1, b1), (c2, b2)]
    mods_off = copy.deepcopy(mods)
    # (a shape whose dgrad is not split over K: the link only arms without a split)
    x = torch.randn(64, 64, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(64, 64, 32, 32, device="cuda")
    extra = torch.randn(64, 64, 32, 32, device="cuda")
    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = _chain(mods, x, g, extra)
    hits, misses = hip_train.bn_dgrad_sums_count(reset=True)
    assert hits == 0 and misses == 1, (hits, misses)
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = _chain(mods_off, x, g, extra)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    torch.cuda.synchronize()
    assert _rel(dx, dx_off) < 1e-2
    for (m, mo) in zip(mods, mods_off):
        for p, q in zip(m[0].parameters(), mo[0].parameters()):
            assert _rel(p.grad, q.grad) < 1e-2
        for p, q in zip(m[1].parameters(), mo[1].parameters()):
            assert _rel(p.grad, q.grad) < 1e-2


@pytest.mark.parametrize("stride", [1, 2])
def test_resnet_stack_with_forks(stride):
    """Two CIFAR BasicBlocks after a stem: the stem BN and block-1 outputs are
    forked (conv1 + shortcut); their sums come from the SECOND consumer's
    dgrad (the one that adds the parked gradient)."""
    from mdistiller_ddp_amd.models.cifar.resnet import BasicBlock
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(4)
    ds = nn.Sequential(nn.Conv2d(64, 128, 1, stride, bias=False), nn.BatchNorm2d(128)) if stride == 2 else None
    net = nn.ModuleList([
        BasicBlock(64, 64, 1, None),
        BasicBlock(64, 128 if stride == 2 else 64, stride, ds),
    ]).cuda().to(memory_format=torch.channels_last)
    stem_c = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    stem_b = nn.BatchNorm2d(64).cuda()
    allm = nn.ModuleList([stem_c, stem_b, net])
    off = copy.deepcopy(allm)
    x = torch.randn(64, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Co = 128 if stride == 2 else 64
    g = torch.randn(64, Co, 16 // stride, 16 // stride, device="cuda").to(torch.bfloat16)

    def run(m):
        sc, sb, blocks = m[0], m[1], m[2]
        xx = x.clone().requires_grad_(True)
        with use_backend("hip"), torch.autocast("cuda", dtype=torch.bfloat16):
            h, _ = hip_train.conv_bn_act_train(xx, sc, sb, "relu", None, False)
            for b in blocks:
                h, _ = b(h)
        h.backward(g)
        torch.cuda.synchronize()
        return h, xx.grad

    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = run(allm)
    hits, _ = hip_train.bn_dgrad_sums_count(reset=True)
    assert hits >= 3, hits
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = run(off)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    assert _rel(out, out_off) < 1e-6
    assert _rel(dx, dx_off) < 2e-2
    for (n, p), (_, q) in zip(allm.named_parameters(), off.named_parameters()):
        assert _rel(p.grad, q.grad) < 2e-2, n


@pytest.mark.parametrize("C,H,stride", [(64, 32, 1), (96, 16, 2), (256, 8, 1)])
def test_depthwise_to_pointwise(C, H, stride):
    """MobileNet pair: depthwise conv + BN + ReLU feeding a pointwise conv; the
    depthwise layer's BN sums come from the pointwise dgrad epilogue."""
    torch.manual_seed(5)
    dw = nn.Conv2d(C, C, 3, stride, 1, groups=C, bias=False).cuda()
    b1 = nn.BatchNorm2d(C).cuda()
    pw = nn.Conv2d(C, 2 * C, 1, bias=False).cuda()
    b2 = nn.BatchNorm2d(2 * C).cuda()
    mods = [(dw, b1), (pw, b2)]
    mods_off = copy.deepcopy(mods)
    x = torch.randn(64, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(64, 2 * C, H // stride, H // stride, device="cuda")
    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = _chain(mods, x, g)
    assert hip_train.bn_dgrad_sums_count(reset=True) == (1, 0)
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = _chain(mods_off, x, g)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    torch.cuda.synchronize()
    torch.testing.assert_close(out, out_off, atol=0, rtol=0)
    assert _rel(dx, dx_off) < 1e-2
    for m, mo in zip(mods, mods_off):
        for p, q in zip(list(m[0].parameters()) + list(m[1].parameters()),
                        list(mo[0].parameters()) + list(mo[1].parameters())):
            assert _rel(p.grad, q.grad) < 1e-2


@pytest.mark.parametrize("C,H,stride,act", [(64, 32, 1, "relu"), (128, 16, 2, "relu"),
                                             (512, 8, 1, "relu"), (96, 14, 1, "relu6")])
def test_pointwise_to_depthwise(C, H, stride, act):
    """MobileNet pair the other way round: pointwise conv + BN + act feeding a
    depthwise conv (the depthwise dgrad takes no BnLink: the pointwise BN runs
    its own backward).  Against an fp32 PyTorch reference, running statistics
    included."""
    torch.manual_seed(6)
    pw = nn.Conv2d(C // 2, C, 1, bias=False).cuda()
    b1 = nn.BatchNorm2d(C).cuda()
    dw = nn.Conv2d(C, C, 3, stride, 1, groups=C, bias=False).cuda()
    b2 = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        for b in (b1, b2):
            b.weight.uniform_(0.5, 1.5)
            b.bias.uniform_(-0.5, 0.5)
    mods_ref = copy.deepcopy([(pw, b1), (dw, b2)])
    x = torch.randn(64, C // 2, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // stride + 1
    g = torch.randn(64, C, Ho, Ho, device="cuda").to(torch.bfloat16).float()
    xx = x.clone().requires_grad_(True)
    h, _ = hip_train.conv_bn_act_train(xx, pw, b1, act, None, False)
    out, _ = hip_train.conv_bn_act_train(h, dw, b2, act, None, False)
    (out.float() * g).sum().backward()
    (r1, rb1), (r2, rb2) = mods_ref
    fa = F.relu if act == "relu" else F.relu6
    x2 = x.float().clone().requires_grad_(True)
    o = fa(rb2(r2(fa(rb1(r1(x2))))))
    o.backward(g)
    torch.cuda.synchronize()
    assert hip_train.slot_errors() == 0
    assert _rel(out.float(), o) < 2e-2
    assert _rel(xx.grad, x2.grad) < 1e-1
    for a, b in zip([pw.weight, b1.weight, b1.bias, dw.weight, b2.weight, b2.bias],
                    [r1.weight, rb1.weight, rb1.bias, r2.weight, rb2.weight, rb2.bias]):
        assert _rel(a.grad, b.grad) < 1e-1
    for b, rb in ((b1, rb1), (b2, rb2)):
        torch.testing.assert_close(b.running_mean, rb.running_mean, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(b.running_var, rb.running_var, rtol=2e-2, atol=2e-2)
        assert int(b.num_batches_tracked) == 1


@pytest.mark.parametrize("inplanes,planes", [(64, 128), (128, 256)])
def test_projection_shortcut_bn_sums_from_bn2(inplanes, planes):
    """A BasicBlock with a projection shortcut: bn2's backward also adds the
    shortcut BN's sums (its output gradient is bn2's dres), so the shortcut
    BN runs the streaming backward -- vs the same block with the links off."""
    from mdistiller_ddp_amd.models.cifar.resnet import BasicBlock
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(6)
    ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, 2, bias=False), nn.BatchNorm2d(planes))
    blk = BasicBlock(inplanes, planes, 2, ds).cuda().to(memory_format=torch.channels_last)
    off = copy.deepcopy(blk)
    # M = 128*16*16: conv2's dgrad runs unsplit, so bn1 also takes its link
    x = torch.randn(128, inplanes, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(128, planes, 16, 16, device="cuda").to(torch.bfloat16)

    def run(m):
        xx = x.clone().requires_grad_(True)
        with use_backend("hip"), torch.autocast("cuda", dtype=torch.bfloat16):
            out, _ = m(xx)
        out.backward(g)
        torch.cuda.synchronize()
        return out, xx.grad

    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = run(blk)
    hits, misses = hip_train.bn_dgrad_sums_count(reset=True)
    assert hits >= 2 and misses == 0, (hits, misses)  # bn1 (from conv2's dgrad) + shortcut BN
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = run(off)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    assert _rel(out, out_off) < 1e-6
    assert _rel(dx, dx_off) < 2e-2
    for (n, p), (_, q) in zip(blk.named_parameters(), off.named_parameters()):
        assert _rel(p.grad, q.grad) < 2e-2, n


@pytest.mark.parametrize("act", ["relu", "none"])
def test_head_bn_sums_from_pool_fc(act):
    """The last BN's output feeds the fused pool + FC head: the head's backward
    adds that BN's sums, so it runs the streaming backward -- vs links off."""
    from mdistiller_ddp_amd.ops.backend import use_backend
    from mdistiller_ddp_amd.ops.nn import conv_bn_act, pool_linear
    torch.manual_seed(7)
    conv = nn.Conv2d(64, 256, 3, 1, 1, bias=False).cuda()
    bn = nn.BatchNorm2d(256).cuda()
    fc = nn.Linear(256, 100).cuda()
    mods = nn.ModuleList([conv, bn, fc])
    off = copy.deepcopy(mods)
    x = torch.randn(128, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(128, 100, device="cuda")

    def run(m):
        xx = x.clone().requires_grad_(True)
        with use_backend("hip"), torch.autocast("cuda", dtype=torch.bfloat16):
            h, _ = conv_bn_act(xx, m[0], m[1], act)
            _, logits = pool_linear(h, m[2])
        logits.float().backward(g)
        torch.cuda.synchronize()
        return logits, xx.grad

    hip_train.bn_dgrad_sums_count(reset=True)
    out, dx = run(mods)
    assert hip_train.bn_dgrad_sums_count(reset=True) == (1, 0)
    hip_train.set_bn_dgrad_sums(False)
    try:
        out_off, dx_off = run(off)
    finally:
        hip_train.set_bn_dgrad_sums(True)
    assert _rel(out, out_off) < 1e-6
    assert _rel(dx, dx_off) < 2e-2
    for (n, p), (_, q) in zip(mods.named_parameters(), off.named_parameters()):
        assert _rel(p.grad, q.grad) < 2e-2, n
