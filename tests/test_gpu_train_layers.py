"""Training-mode conv + BN (+res) (+ReLU) native kernels vs PyTorch fp32:
forward values, running statistics, and gradients of x, weight, gamma,
beta and the residual."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import hip_train

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, Cin, H, Cout, k, stride, pad, x_grad
    (16, 3, 32, 32, 3, 1, 1, False),    # stem (input padded to 8 channels)
    (4, 3, 56, 64, 7, 2, 3, False),     # ImageNet 7x7/s2 stem
    (16, 32, 32, 64, 3, 1, 1, True),
    (16, 64, 32, 64, 3, 1, 1, True),
    (16, 64, 32, 128, 3, 2, 1, True),   # stride 2 dgrad
    (16, 128, 16, 256, 3, 2, 1, True),
    (16, 64, 32, 128, 1, 2, 0, True),   # 1x1 shortcut
    (16, 256, 8, 256, 3, 1, 1, True),
    (16, 128, 16, 128, 3, 1, 1, True),  # halo weight gradient, 16-wide rows
    (8, 16, 32, 16, 3, 1, 1, True),     # vec8 loaders (resnet20 widths)
    (4, 24, 15, 40, 3, 2, 1, True),
]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act,with_res", [("relu", True), ("relu", False), ("none", False)])
def test_conv_bn_act_train(shape, act, with_res):
    N, Cin, H, Cout, k, s, p, xg = shape
    torch.manual_seed(0)
    conv = nn.Conv2d(Cin, Cout, k, s, p, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    # ours
    x1 = x.clone().requires_grad_(xg)
    r1 = res.clone().requires_grad_(True) if with_res else None
    assert hip_train.train_supported(x1, conv, bn)
    out, pre = hip_train.conv_bn_act_train(x1, conv, bn, act, r1, True)
    # incoming gradients are bf16 tensors in the native path; give the fp32
    # reference the same rounded values
    g = torch.randn_like(out.float()).to(torch.bfloat16).float()
    gp = (torch.randn_like(out.float()) * 0.1).to(torch.bfloat16).float()
    torch.autograd.backward([out.float(), pre.float()], [g, gp])
    # reference (fp32 on the same bf16 inputs)
    x2 = x.float().clone().requires_grad_(xg)
    r2 = res.float().clone().requires_grad_(True) if with_res else None
    z = bn_r(conv_r(x2))
    if with_res:
        z = z + r2
    o = F.relu(z) if act == "relu" else z
    torch.autograd.backward([o, z], [g, gp])
    tol = 4e-2
    torch.testing.assert_close(out.float(), o, atol=tol, rtol=tol)
    torch.testing.assert_close(pre.float(), z, atol=tol, rtol=tol)
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, bn_r.running_var, atol=1e-2, rtol=1e-2)

    def rel(a, b):
        return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()

    # per-channel sums over N*H*W terms that largely cancel: bf16 storage of y
    # flips a few ReLU-mask decisions near z = 0, hence the looser bound
    assert rel(bn.weight.grad, bn_r.weight.grad) < 5e-2
    assert rel(bn.bias.grad, bn_r.bias.grad) < 5e-2
    assert rel(conv.weight.grad, conv_r.weight.grad) < 5e-2
    if xg:
        assert rel(x1.grad, x2.grad) < 5e-2
    if with_res:
        assert rel(r1.grad, r2.grad) < 5e-2


@pytest.mark.parametrize("shape", SHAPES)
def test_dgrad_wgrad_kernels_exact_inputs(shape):
    """The MFMA dgrad / wgrad kernels alone, on bf16 inputs given to both sides."""
    N, Cin, H, Cout, k, s, p, xg = shape
    torch.manual_seed(1)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, k, k, device="cuda") * 0.1).to(torch.bfloat16).float()
    Ho = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16)
    xr = x.float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=s, padding=p).backward(dy.float())
    dw = hip_train.conv_wgrad(x, dy, tuple(w.shape), s, p)
    rel_w = ((dw - wr.grad).norm() / wr.grad.norm()).item()
    assert rel_w < 1e-2, rel_w
    if Cout % 8 == 0:
        dx = hip_train.conv_dgrad(dy, w, tuple(x.shape), s, p)
        rel_x = ((dx.float() - xr.grad).norm() / xr.grad.norm()).item()
        assert rel_x < 1e-2, rel_x


@pytest.mark.parametrize("name", ["resnet8x4", "wrn_16_2", "vgg8", "MobileNetV2", "ShuffleV1", "ShuffleV2",
                                  "tiny_MobileNetV2", "tiny_ShuffleV2"])
def test_student_train_step_uses_native_path(name):
    """A full student training forward/backward through the native path vs an
    fp32 PyTorch reference: its gradient error must be in the same band as the
    stock bf16 (MIOpen) path's, and so must every BN's running statistics
    (Tiny-ImageNet MobileNetV2: depthwise convs with biases, folded into the
    following training BN)."""
    from mdistiller_ddp_amd.models import cifar_model_dict, tiny_imagenet_model_dict
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(0)
    tiny = name.startswith("tiny_")
    table, hw, ncls = (tiny_imagenet_model_dict, 64, 200) if tiny else (cifar_model_dict, 32, 100)
    m1 = table[name[5:] if tiny else name][0](num_classes=ncls).cuda().to(memory_format=torch.channels_last)
    m2 = copy.deepcopy(m1)
    m3 = copy.deepcopy(m1)
    x = torch.randn(32, 3, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (32,), device="cuda")
    grads = []
    for m, be, amp in ((m1, "hip", True), (m2, "torch", True), (m3, "torch", False)):
        with use_backend(be), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            logits, _ = m(x)
            loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        grads.append(torch.cat([p.grad.float().reshape(-1) for p in m.parameters()]))
    ref = grads[2]
    e_native = ((grads[0] - ref).norm() / ref.norm()).item()
    e_miopen = ((grads[1] - ref).norm() / ref.norm()).item()
    assert e_native < max(2.0 * e_miopen, 0.05), (e_native, e_miopen)
    rm = [torch.cat([b.float().reshape(-1) for n, b in m.named_buffers() if "running" in n])
          for m in (m1, m2, m3)]
    r_native = ((rm[0] - rm[2]).norm() / rm[2].norm()).item()
    r_miopen = ((rm[1] - rm[2]).norm() / rm[2].norm()).item()
    assert r_native < max(2.0 * r_miopen, 1e-2), (r_native, r_miopen)


@pytest.mark.parametrize("student", ["resnet8x4", "MobileNetV2"])
def test_pack_cache_matches_per_layer_packing(student):
    """TrainStep with the one-launch PackCache == per-layer packing, over a few
    steps (the packed weights must track every optimizer update; MobileNetV2's
    depthwise weights ride in the same launch)."""
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.SOLVER.LR = 0.005  # a random teacher's KD steps at 0.05 are chaotic (tiny diffs blow up)
    torch.manual_seed(0)
    d1 = build_distiller(cfg, 100, "cuda")
    d2 = copy.deepcopy(d1)
    init = None
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    out = []
    for d, use_cache in ((d1, True), (d2, False)):
        d.train()
        st = TrainStep(d, cfg, "cuda", use_graph=False, dtype=torch.bfloat16)
        st.set_epoch(1.0)
        if init is None:
            init = st.flat.data.clone()
        if not use_cache:
            st._packs = hip_train.PackCache()
            st._packs.pack_all = lambda device, **kw: False
        for b in SyntheticLoader("cifar100", 16, "cuda", steps_per_epoch=4, channels_last=True):
            st.step(b)
        torch.cuda.synchronize()
        if use_cache:
            assert st._packs.entries and st._packs._table is not None
            if student == "MobileNetV2":
                assert any(e["meta"][1] < 0 for e in st._packs.entries.values())
        out.append(st.flat.data.clone())
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    if student == "resnet8x4":
        torch.testing.assert_close(out[0], out[1], rtol=0, atol=0)
    else:
        # MobileNetV2's 12-channel layers and its classifier run on MIOpen /
        # hipBLASLt, which are not guaranteed bitwise reproducible even in
        # deterministic mode; stale packs would put an error of the order of the
        # steps' own movement
        moved = (out[1] - init).norm()
        rel = ((out[0] - out[1]).norm() / moved).item()
        assert moved.item() > 0 and rel < 1e-3, rel


@pytest.mark.parametrize("shapes", [
    [(64, 3, 3, 3), (64, 64, 3, 3), (128, 64, 1, 1), (256, 128, 3, 3)],
    [(64, 3, 7, 7), (32, 24, 3, 3), (40, 72, 1, 1), (512, 512, 3, 3), (24, 8, 5, 5)],
])
def test_pack_multi_equals_per_layer_pack(shapes):
    """The one-launch tiled multi-layer pack writes exactly what the per-layer
    pack writes (both operand layouts, padding untouched and zero)."""
    torch.manual_seed(0)
    cache = hip_train.PackCache()
    ref, bufs = [], []
    for (co, ci, kh, kw) in shapes:
        w = torch.randn(co, ci, kh, kw, device="cuda")
        wf_r, wt_r, Kp, KpT = hip_train.pack_weights(w, True)
        ref.append((wf_r, wt_r))
        # registration-time pack (zeros the padding), then scribble the live part
        wf, wt, _, _ = hip_train.pack_weights(w, True)
        K, KT = kh * kw * ci, kh * kw * co
        wf[:, :K] = 7.0
        wt[:, :KT] = 7.0
        cache.entries[id(w)] = dict(weight=w, wf=wf, wt=wt, meta=(co, ci, kh, kw, Kp, KpT))
        bufs.append((w, wf, wt))
    cache._dirty = True
    assert cache.pack_all(torch.device("cuda"))
    torch.cuda.synchronize()
    for (wf_r, wt_r), (_, wf, wt) in zip(ref, bufs):
        assert torch.equal(wf, wf_r)
        assert torch.equal(wt, wt_r)


def test_wrn_convs_take_native_training_path():
    """Pre-activation WRN: every conv (no BN after it) and every BN+ReLU of a
    training forward dispatches to the native kernels."""
    from mdistiller_ddp_amd.models import cifar_model_dict
    from mdistiller_ddp_amd.ops.backend import use_backend
    calls = {"conv": 0, "bn": 0}
    orig_c, orig_b = hip_train.conv_act_train, hip_train.bn_act_train

    def cc(*a, **k):
        calls["conv"] += 1
        return orig_c(*a, **k)

    def cb(*a, **k):
        calls["bn"] += 1
        return orig_b(*a, **k)

    hip_train.conv_act_train, hip_train.bn_act_train = cc, cb
    try:
        m = cifar_model_dict["wrn_16_2"][0](num_classes=100).cuda().to(memory_format=torch.channels_last)
        x = torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
        with use_backend("hip"), torch.autocast("cuda", dtype=torch.bfloat16):
            logits, _ = m(x)
        logits.float().sum().backward()
    finally:
        hip_train.conv_act_train, hip_train.bn_act_train = orig_c, orig_b
    n_conv = sum(1 for mod in m.modules() if isinstance(mod, nn.Conv2d))
    n_bn = sum(1 for mod in m.modules() if isinstance(mod, nn.BatchNorm2d))
    assert calls["conv"] == n_conv - sum(1 for b in m.modules() if hasattr(b, "bn2")), calls
    assert calls["bn"] == n_bn - sum(1 for b in m.modules() if hasattr(b, "bn2")), calls


GROUPED = [(8, 240, 16, 120, 3, False, 1, 1), (8, 120, 8, 480, 3, True, 1, 1),
           (4, 480, 8, 240, 3, False, 1, 1), (8, 64, 16, 32, 2, True, 1, 1),
           (64, 72, 16, 240, 3, True, 1, 1),      # ShuffleV1 conv3 (24 -> 80 per group, padded)
           (64, 240, 16, 72, 3, False, 1, 1),     # ShuffleV1 conv1 (80 -> 24 per group)
           (16, 48, 16, 96, 2, False, 3, 2)]      # 3x3 stride-2 grouped (strided grouped dgrad)


@pytest.mark.parametrize("N,Cin,H,Cout,G,with_res,k,s", GROUPED)
@pytest.mark.parametrize("compact", [True, False])
def test_grouped_conv_bn_act_train(N, Cin, H, Cout, G, with_res, k, s, compact):
    """Grouped conv (ShuffleNetV1) + BN (+res) + ReLU on the native path -- the
    compact per-group GEMM (group-aligned tiles, default) and the dense
    block-diagonal GEMM -- vs fp32 PyTorch: outputs, running stats, all gradients."""
    torch.manual_seed(2)
    conv = nn.Conv2d(Cin, Cout, k, s, k // 2, groups=G, bias=False).cuda()
    bn = nn.BatchNorm2d(Cout).cuda()
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(N, Cin, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * (k // 2) - k) // s + 1
    res = torch.randn(N, Cout, Ho, Ho, device="cuda").to(torch.bfloat16) if with_res else None
    x1 = x.clone().requires_grad_(True)
    r1 = res.clone().requires_grad_(True) if with_res else None
    hip_train.set_grouped_native(True)
    hip_train.set_grouped_compact(compact)
    try:
        assert hip_train.train_supported(x1, conv, bn)
        out, _ = hip_train.conv_bn_act_train(x1, conv, bn, "relu", r1, False)
    finally:
        hip_train.set_grouped_native(False)
        hip_train.set_grouped_compact(True)
    g = torch.randn_like(out.float()).to(torch.bfloat16).float()
    out.float().backward(g)
    x2 = x.float().clone().requires_grad_(True)
    r2 = res.float().clone().requires_grad_(True) if with_res else None
    z = bn_r(conv_r(x2))
    if with_res:
        z = z + r2
    F.relu(z).backward(g)
    torch.testing.assert_close(out.float(), F.relu(z), atol=4e-2, rtol=4e-2)
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, atol=1e-3, rtol=1e-3)

    def rel(a, b):
        return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()

    assert conv.weight.grad.shape == conv_r.weight.grad.shape
    assert rel(conv.weight.grad, conv_r.weight.grad) < 5e-2
    assert rel(x1.grad, x2.grad) < 5e-2
    assert rel(bn.weight.grad, bn_r.weight.grad) < 5e-2
    if with_res:
        assert rel(r1.grad, r2.grad) < 5e-2


def test_pack_multi_depthwise_rows_equal_dw_pack():
    """Depthwise rows of the multi-layer pack == the per-layer dw pack."""
    torch.manual_seed(0)
    cache = hip_train.PackCache()
    ws, outs = [], []
    for C in (16, 96, 480, 1024):
        w = torch.randn(C, 1, 3, 3, device="cuda")
        wp = torch.full((9, C), 7.0, device="cuda")
        cache.register_dw(w, wp)
        ws.append(w)
        outs.append(wp)
    w2 = torch.randn(64, 32, 3, 3, device="cuda")  # a dense layer in the same launch
    wf, wt, Kp, KpT = hip_train.pack_weights(w2, True)
    cache.register(w2, wf, wt, 64, 32, 3, 3, Kp, KpT)
    assert cache.pack_all(torch.device("cuda"))
    torch.cuda.synchronize()
    for w, wp in zip(ws, outs):
        assert torch.equal(wp, hip_train.dw_pack(w))
    wf_r, wt_r, _, _ = hip_train.pack_weights(w2, True)
    assert torch.equal(wf, wf_r) and torch.equal(wt, wt_r)


@pytest.mark.parametrize("student", ["resnet8x4", "resnet20"])
def test_wgrad_bn_fused_launch_matches_separate(student):
    """mda_conv_wgrad_nored_bn: under the captured backward each deferred
    weight-gradient GEMM rides in the launch of the next BN-backward apply.
    The fused launch runs the same two kernel bodies, so a graph-replayed
    training run matches the unfused one to the BN-sum atomics' run-to-run
    spread, and the fused path actually ran."""
    import copy
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.SOLVER.LR = 0.005
    torch.manual_seed(0)
    d0 = build_distiller(cfg, 100, "cuda")
    batches = list(SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=8, channels_last=True))
    out = []
    for fuse in (True, False, False):
        hip_train.set_wgrad_bn_fuse(fuse)
        try:
            d = copy.deepcopy(d0)
            d.train()
            st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
            st.set_epoch(1.0)
            n0 = hip_train._WG_FUSE_COUNT[0]
            for b in batches:
                st.step(b)
            torch.cuda.synchronize()
            fused = hip_train._WG_FUSE_COUNT[0] - n0
        finally:
            hip_train.set_wgrad_bn_fuse(True)
        out.append((st.flat.data.clone(), fused))
    (p1, n1), (p2, n2), (p3, n3) = out
    assert n1 > 0 and n2 == 0 and n3 == 0, (n1, n2, n3)
    assert torch.isfinite(p1).all()
    spread = ((p3 - p2).norm() / p2.norm()).item()
    rel = ((p1 - p2).norm() / p2.norm()).item()
    assert rel <= 3 * spread + 1e-4, (rel, spread)


@pytest.mark.parametrize("student", ["resnet8x4", "resnet20"])
def test_apply_ride_matches_separate(student):
    """mda_conv1x1_bnacc_apply: a residual block's conv1 BN apply rides in the
    launch of its projection shortcut's 1x1 conv.  Same kernel bodies as the
    two separate launches, so graph-replayed training matches the unfused
    path to the BN-sum atomics' run-to-run spread, and the fused path ran."""
    import copy
    from mdistiller_ddp_amd.config import get_cfg
    from mdistiller_ddp_amd.engine.build import build_distiller
    from mdistiller_ddp_amd.engine.step import TrainStep
    from mdistiller_ddp_amd.data.synthetic import SyntheticLoader
    cfg = get_cfg()
    cfg.DISTILLER.TYPE = "KD"
    cfg.DISTILLER.TEACHER = "resnet32x4"
    cfg.DISTILLER.STUDENT = student
    cfg.DISTILLER.RANDOM_TEACHER = True
    cfg.SOLVER.LR = 0.005
    torch.manual_seed(0)
    d0 = build_distiller(cfg, 100, "cuda")
    batches = list(SyntheticLoader("cifar100", 64, "cuda", steps_per_epoch=8, channels_last=True))
    out = []
    for ride in (True, False, False):
        hip_train.set_apply_ride(ride)
        try:
            d = copy.deepcopy(d0)
            d.train()
            st = TrainStep(d, cfg, "cuda", use_graph=True, dtype=torch.bfloat16)
            st.set_epoch(1.0)
            n0 = hip_train._RIDE_COUNT[0]
            for b in batches:
                st.step(b)
            torch.cuda.synchronize()
            n = hip_train._RIDE_COUNT[0] - n0
        finally:
            hip_train.set_apply_ride(True)
        out.append((st.flat.data.clone(), n))
    (p1, n1), (p2, n2), (p3, n3) = out
    assert n1 > 0 and n2 == 0 and n3 == 0, (n1, n2, n3)
    assert torch.isfinite(p1).all()
    spread = ((p3 - p2).norm() / p2.norm()).item()
    rel = ((p1 - p2).norm() / p2.norm()).item()
    # the fused launch runs small shortcuts (M < 16384) on the streaming 1x1
    # kernel, the separate path on the implicit-GEMM one: another summation
    # order (resnet20: 7.5e-4 after 8 steps, the separate runs bitwise equal)
    assert rel <= 3 * spread + 2e-3, (rel, spread)
