"""HIP kernels vs plain-PyTorch fp32 references: fused CE/KD/DKD losses and
the flat optimizers (SGD, Adam, AdamW, DOT, grad-norm clip)."""
import pytest
import torch

from mdistiller_ddp_amd.ops import losses as L
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_grads(fn, s, *args):
    s = s.detach().float().clone().requires_grad_(True)
    ce, kd = fn(s, *args)
    gce, = torch.autograd.grad(ce, s, retain_graph=True)
    gkd, = torch.autograd.grad(kd, s)
    return ce.detach(), kd.detach(), gce, gkd


def _hip_grads(fn, s, *args):
    s = s.detach().clone().requires_grad_(True)
    with use_backend("hip"):
        ce, kd = fn(s, *args)
    gce, = torch.autograd.grad(ce, s, retain_graph=True)
    gkd, = torch.autograd.grad(kd, s)
    return ce.detach(), kd.detach(), gce.float(), gkd.float()


@pytest.mark.parametrize("B,C", [(64, 100), (7, 1000), (130, 200), (3, 37)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ce_kd(B, C, dtype):
    torch.manual_seed(0)
    s = (torch.randn(B, C, device=DEV) * 3).to(dtype)
    t = (torch.randn(B, C, device=DEV) * 3).to(dtype)
    y = torch.randint(0, C, (B,), device=DEV)

    def ref(s_, t_, y_):
        return 0.1 * L.cross_entropy(s_, y_), 0.9 * L.kd_loss_ref(s_, t_.float(), 4.0)

    def hip(s_, t_, y_):
        return L.ce_kd(s_, t_, y_, 4.0, 0.1, 0.9)

    r = _ref_grads(ref, s, t, y)
    h = _hip_grads(hip, s, t, y)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b in zip(h, r):
        torch.testing.assert_close(a, b, atol=tol * max(1.0, b.abs().max().item()), rtol=tol)


@pytest.mark.parametrize("B,C,gap,T", [(64, 100, 5.0, 4.0), (9, 1000, 5.0, 4.0), (33, 200, 5.0, 4.0),
                                       (16, 1000, 150.0, 1.0), (16, 100, 400.0, 4.0)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_ce_dkd(B, C, gap, T, dtype):
    """Includes near-one-hot teachers (target gap >> 88 at T): the non-target
    softmax must be normalised by its own maximum, as the reference's
    -1000*gt_mask does, or every non-target probability underflows."""
    torch.manual_seed(1)
    s = (torch.randn(B, C, device=DEV) * 3).to(dtype)
    t = (torch.randn(B, C, device=DEV) * 3).to(dtype)
    y = torch.randint(0, C, (B,), device=DEV)
    t[torch.arange(B), y] += gap  # confident teacher

    def ref(s_, t_, y_):
        return L.cross_entropy(s_, y_), L.dkd_loss_ref(s_, t_.float(), y_, 1.0, 8.0, T)

    def hip(s_, t_, y_):
        return L.ce_dkd(s_, t_, y_, 1.0, 1.0, 8.0, T)

    r = _ref_grads(ref, s, t, y)
    h = _hip_grads(hip, s, t, y)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b in zip(h, r):
        torch.testing.assert_close(a, b, atol=tol * max(1.0, b.abs().max().item()), rtol=tol)


def _flat_pair(n_params=(1000, 37, 4096)):
    from mdistiller_ddp_amd.engine.optim import FlatParams
    torch.manual_seed(2)
    out = []
    for _ in range(2):
        ps = [torch.nn.Parameter(torch.randn(n, device=DEV)) for n in n_params]
        out.append(ps)
    for a, b in zip(*out):
        b.data.copy_(a.data)
    return out


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw", "sgd_clip", "dot"])
def test_optimizers_hip_vs_torch(kind):
    from mdistiller_ddp_amd.engine.optim import FlatParams, FlatSGD, FlatAdam, FlatDOT
    pa, pb = _flat_pair()
    flats = []
    for ps, be in ((pa, "hip"), (pb, "torch")):
        with use_backend(be):
            f = FlatParams(ps, 2 if kind == "dot" else 1)
            if kind == "sgd":
                o = FlatSGD(f, 0.1, 0.9, 5e-4, grad_scale=0.5)
            elif kind == "sgd_clip":
                o = FlatSGD(f, 0.1, 0.9, 5e-4, grad_clip=0.3)
            elif kind == "adam":
                o = FlatAdam(f, 1e-3, weight_decay=1e-2)
            elif kind == "adamw":
                o = FlatAdam(f, 1e-3, weight_decay=1e-2, decoupled=True)
            else:
                o = FlatDOT(f, 0.1, 0.825, 0.975, 5e-4)
                o.set_reachability([True, True, False], [True, False, True])
        flats.append((f, o))
    torch.manual_seed(3)
    for it in range(4):
        g = torch.randn_like(flats[0][0].grads)
        for f, o in flats:
            f.grads.copy_(g)
            o.set_lr(0.1 / (it + 1))
            o.step()
    torch.testing.assert_close(flats[0][0].data, flats[1][0].data, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("shape_s,shape_t", [((8, 64, 32, 32), (8, 256, 32, 32)),
                                             ((4, 16, 8, 8), (4, 48, 8, 8)),
                                             ((3, 32, 56, 56), (3, 64, 56, 56))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_at_loss_kernel(shape_s, shape_t, dtype):
    from mdistiller_ddp_amd.ops import feat_losses as FL
    torch.manual_seed(4)
    fs = torch.randn(*shape_s, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    ft = torch.randn(*shape_t, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    a = fs.clone().requires_grad_(True)
    with use_backend("hip"):
        l1 = FL.single_stage_at_loss(a, ft, 2)
    l1.backward()
    b = fs.float().clone().requires_grad_(True)
    l2 = FL.single_stage_at_loss_ref(b, ft.float(), 2)
    l2.backward()
    tol = 1e-4 if dtype == torch.float32 else 3e-2
    torch.testing.assert_close(l1.float(), l2, rtol=tol, atol=1e-7)
    torch.testing.assert_close(a.grad.float(), b.grad, rtol=tol, atol=tol * b.grad.abs().max().item())


@pytest.mark.parametrize("N,C,H", [(8, 64, 8), (16, 256, 4), (3, 24, 5)])
def test_ofd_fused_loss_matches_torch(N, C, H):
    import importlib
    ofd_mod = importlib.import_module("mdistiller_ddp_amd.distillers.OFD")
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(7)
    s = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    m = -torch.rand(1, C, 1, 1, device="cuda")
    sh = s.clone().requires_grad_(True)
    with use_backend("hip"):
        assert ofd_mod._ofd_native_ok(sh, t)
        l = ofd_mod.feat_loss(sh, t, m)
    (l * 0.5).backward()
    sr = s.float().clone().requires_grad_(True)
    with use_backend("torch"):
        lr = ofd_mod.feat_loss(sr, t.float(), m)
    (lr * 0.5).backward()
    torch.testing.assert_close(l, lr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(sh.grad.float(), sr.grad, rtol=2e-2, atol=1e-4)


@pytest.mark.parametrize("mode", ["ce", "kd", "dkd"])
def test_unit_seed_backward_matches_scaled_path(mode):
    """With the training step's registered unit seeds the loss backward
    returns the kernel's stored (summed) gradient without a launch; it must
    equal the go * g path of an ordinary seed to within one bf16 rounding."""
    torch.manual_seed(0)
    B, C = 64, 100
    s0 = torch.randn(B, C, device="cuda").to(torch.bfloat16)
    t = torch.randn(B, C, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, C, (B,), device="cuda")
    unit = torch.ones((), device="cuda")
    L.register_unit_seed(unit)
    grads = []
    for seed in (unit, torch.ones((), device="cuda")):
        s = s0.clone().requires_grad_(True)
        with use_backend("hip"):
            if mode == "ce":
                terms = [L.ce(s, y, 1.0)]
            elif mode == "kd":
                terms = list(L.ce_kd(s, t, y, 4.0, 0.1, 0.9))
            else:
                terms = list(L.ce_dkd(s, t, y, 1.0, 1.0, 8.0, 4.0))
        torch.autograd.backward(terms, [seed] * len(terms))
        grads.append(s.grad.float())
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-2, atol=1e-5)
