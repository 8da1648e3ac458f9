"""Fused training BN (csrc/bn.hip "fused BN", csrc/bnslot.h): the region-based
conv+stats -> apply-with-finalize forward and the one-launch grid-barrier
backward vs an fp32 PyTorch reference, vs the unfused partial-rows path, under
hipGraph replay with the per-step arena of one-shot regions, and no barrier timeouts."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_train

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, Cin, H, Cout, k, stride, pad
    (64, 64, 32, 64, 3, 1, 1),    # flagship stage 1: the HOLD<8> backward
    (64, 128, 16, 128, 3, 1, 1),  # HOLD<4>
    (64, 256, 8, 256, 3, 1, 1),   # HOLD<2>, 4 slot shards
    (32, 64, 56, 64, 3, 1, 1),    # M = 100k: re-reading backward (no HOLD)
    (8, 512, 7, 1024, 1, 1, 0),   # 1 slot shard
    (4, 24, 15, 40, 3, 2, 1),     # C/8 not a power of two
]


def _ref(conv, bn, x, res, act):
    z = bn(conv(x))
    if res is not None:
        z = z + res
    return (F.relu(z) if act == "relu" else z), z


def _run(conv, bn, x, res, act, g, gp):
    x1 = x.clone().requires_grad_(True)
    r1 = res.clone().requires_grad_(True) if res is not None else None
    out, pre = hip_train.conv_bn_act_train(x1, conv, bn, act, r1, True)
    torch.autograd.backward([out.float(), pre.float()], [g, gp])
    return out, pre, x1.grad, (r1.grad if r1 is not None else None)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("with_res", [True, False])
def test_fused_matches_fp32_and_unfused(shape, with_res):
    N, Cin, H, Cout, k, s, p = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_u, bn_u = copy.deepcopy(conv), copy.deepcopy(bn)
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    g = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16).float()
    gp = (torch.randn(N, Cout, Ho, Ho, device="cuda") * 0.1).to(torch.bfloat16).float()

    hip_train.set_bn_fused(True)
    out, pre, dx, dr = _run(conv, bn, x, res, "relu", g, gp)
    hip_train.set_bn_fused(False)
    try:
        out_u, pre_u, dx_u, dr_u = _run(conv_u, bn_u, x, res, "relu", g, gp)
    finally:
        hip_train.set_bn_fused(True)
    torch.cuda.synchronize()
    assert hip_train.slot_errors() == 0

    x2 = x.float().clone().requires_grad_(True)
    r2 = res.float().clone().requires_grad_(True) if with_res else None
    o, z = _ref(conv_r, bn_r, x2, r2, "relu")
    torch.autograd.backward([o, z], [g, gp])

    def rel(a, b):
        return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

    # vs fp32
    torch.testing.assert_close(out.float(), o, atol=4e-2, rtol=4e-2)
    torch.testing.assert_close(pre.float(), z, atol=4e-2, rtol=4e-2)
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, bn_r.running_var, atol=1e-2, rtol=1e-2)
    assert int(bn.num_batches_tracked) == 1
    assert rel(bn.weight.grad, bn_r.weight.grad) < 5e-2
    assert rel(bn.bias.grad, bn_r.bias.grad) < 5e-2
    assert rel(conv.weight.grad, conv_r.weight.grad) < 5e-2
    assert rel(dx, x2.grad) < 5e-2
    if with_res:
        assert rel(dr, r2.grad) < 5e-2
    # vs the unfused native path: same bf16 roundings, fp64 vs fp64 sums
    assert rel(out, out_u) < 1e-3
    assert rel(bn.weight.grad, bn_u.weight.grad) < 1e-3
    assert rel(bn.bias.grad, bn_u.bias.grad) < 1e-3
    assert rel(dx, dx_u) < 1e-2
    torch.testing.assert_close(bn.running_var, bn_u.running_var, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("C", [64, 256, 2048])
def test_standalone_bn_act_train(C):
    """bn_act_train (pre-activation BN / depthwise path): stats pass into the
    slot + apply-with-finalize, fused backward with the residual gradient."""
    torch.manual_seed(1)
    N, H = 16, 8
    bn = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_r = copy.deepcopy(bn)
    x = (torch.randn(N, C, H, H, device="cuda") * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x)
    x1, r1 = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
    out, _ = hip_train.bn_act_train(x1, bn, "relu", r1, False)
    g = torch.randn_like(out.float()).to(torch.bfloat16).float()
    out.float().backward(g)
    x2, r2 = x.float().requires_grad_(True), res.float().requires_grad_(True)
    o = F.relu(bn_r(x2) + r2)
    o.backward(g)
    torch.cuda.synchronize()
    assert hip_train.slot_errors() == 0
    torch.testing.assert_close(out.float(), o, atol=4e-2, rtol=4e-2)
    for a, b in ((x1.grad, x2.grad), (r1.grad, r2.grad), (bn.weight.grad, bn_r.weight.grad),
                 (bn.bias.grad, bn_r.bias.grad)):
        assert ((a.float() - b).norm() / b.norm()).item() < 5e-2


def test_arena_regions_graph_replay_matches_eager():
    """Inside a training step every BN call takes a one-shot region of the
    per-device arena, zeroed by one memset at the step start; a captured graph
    of that step (memset + conv/BN forward + fused backward) replays to the
    eager values, run after run, and matches the out-of-step fallback regions."""
    torch.manual_seed(2)
    dev = torch.device("cuda")
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).cuda()
    bn = nn.BatchNorm2d(64).cuda()
    conv2 = nn.Conv2d(64, 128, 3, 2, 1, bias=False).cuda()
    bn2 = nn.BatchNorm2d(128).cuda()
    x = torch.randn(32, 64, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(32, 128, 8, 8, device="cuda").to(torch.bfloat16)
    xs = x.clone().requires_grad_(True)
    params = (xs, conv.weight, bn.weight, bn.bias, conv2.weight, bn2.weight, bn2.bias)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())

    def body(step):
        for t in params:
            t.grad = None
        if step:
            hip_train.bn_step_begin(dev)
        h, _ = hip_train.conv_bn_act_train(xs, conv, bn, "relu", None, False)
        out, _ = hip_train.conv_bn_act_train(h, conv2, bn2, "relu", None, False)
        out.backward(g)
        if step:
            hip_train.bn_step_end(dev)
        return out

    with torch.cuda.stream(s):
        ref_out = body(False).detach().clone()       # fallback regions (torch.zeros per call)
        ref = [t.grad.detach().clone() for t in params]
        arena_out = body(True).detach().clone()      # arena regions, eager
        arena = [t.grad.detach().clone() for t in params]
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            out_g = body(True)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(arena_out, ref_out, atol=0, rtol=0)
    for a, r in zip(arena, ref):
        torch.testing.assert_close(a, r, atol=1e-6, rtol=1e-5)
    for _ in range(3):
        gr.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out_g, ref_out, atol=0, rtol=0)
        for t, r in zip(params, ref):
            torch.testing.assert_close(t.grad, r, atol=1e-6, rtol=1e-5)
    assert hip_train.slot_errors() == 0


@pytest.mark.parametrize("inplanes,planes,stride", [(64, 64, 1), (64, 128, 2)])
@pytest.mark.parametrize("branch", [True, False])
def test_residual_block_grad_fork(inplanes, planes, stride, branch):
    """A CIFAR BasicBlock on the native path: x's two consumers (conv1 and the
    identity / projection shortcut) sum their input gradients in the second
    consumer's dgrad epilogue (GradFork), the projection running on the
    branch stream -- vs the same native block with autograd's add (tight) and
    vs the fp32 PyTorch block (bf16 band)."""
    from mdistiller_ddp_amd.models.cifar.resnet import BasicBlock
    from mdistiller_ddp_amd.ops import nn as mda_nn
    from mdistiller_ddp_amd.ops.backend import use_backend
    from mdistiller_ddp_amd.runtime import streams
    torch.manual_seed(3)
    ds = None
    if stride != 1 or inplanes != planes:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    blk = BasicBlock(inplanes, planes, stride, ds).cuda().to(memory_format=torch.channels_last)
    blk_nf, ref = copy.deepcopy(blk), copy.deepcopy(blk)
    x = torch.randn(32, inplanes, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(32, planes, 16 // stride, 16 // stride, device="cuda").to(torch.bfloat16)

    def run(m, forks):
        mda_nn.set_grad_forks(forks)
        prev = streams.branches_enabled()
        streams.set_branches(branch)
        try:
            xx = x.clone().requires_grad_(True)
            with use_backend("hip"), torch.autocast("cuda", dtype=torch.bfloat16):
                out, _ = m(xx)
            out.backward(g)
            torch.cuda.current_stream().wait_stream(streams.branch_stream(x.device))
        finally:
            mda_nn.set_grad_forks(True)
            streams.set_branches(prev)
        return out, xx.grad

    out, dx = run(blk, True)
    out_nf, dx_nf = run(blk_nf, False)
    x2 = x.float().clone().requires_grad_(True)
    with use_backend("torch"):
        o2, _ = ref(x2)
    o2.backward(g.float())
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(dx, dx_nf) < 1e-2
    for (n, p), (_, q) in zip(blk.named_parameters(), blk_nf.named_parameters()):
        assert rel(p.grad, q.grad) < 1e-2, n
    assert rel(out, o2) < 2e-2
    assert rel(dx, x2.grad) < 1e-1
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert rel(p.grad, q.grad) < 1e-1, n
