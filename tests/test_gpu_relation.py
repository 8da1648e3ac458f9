"""SP / PKT / RKD on the batch Gram (csrc/relation.hip) vs the PyTorch fp32 forms.

The native kernels read bf16 features; the reference runs the PyTorch form
(`ops/feat_losses.py::*_ref`, line-for-line the reference distillers) in fp32 on
the same bf16-rounded values, so only summation order and the bf16 gradient
store differ.
"""
import pytest
import torch

from mdistiller_ddp_amd.ops import feat_losses as FL
from mdistiller_ddp_amd.ops import _ext

pytestmark = pytest.mark.gpu


def _feat(shape, cl, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    f = (torch.randn(shape, device="cuda", generator=g) * scale).to(torch.bfloat16)
    if cl and f.dim() == 4:
        f = f.contiguous(memory_format=torch.channels_last)
    return f


def _run(fn_native, fn_ref, f_s, f_t):
    a = f_s.clone().requires_grad_(True)
    ln = fn_native(a, f_t)
    ln.sum().backward()
    b = f_s.detach().float().clone().requires_grad_(True)
    lr = fn_ref(b, f_t.float())
    lr.sum().backward()
    torch.cuda.synchronize()
    return ln.detach().float(), lr.detach().float(), a.grad.float(), b.grad.float()


def _check(ln, lr, gn, gr, tol_l=2e-3, tol_g=2e-2):
    assert torch.isfinite(ln).all() and torch.isfinite(gn).all()
    rel_l = ((ln - lr).abs() / lr.abs().clamp_min(1e-12)).max().item()
    rel_g = ((gn - gr).norm() / gr.norm().clamp_min(1e-20)).item()
    assert rel_l < tol_l, (ln, lr)
    assert rel_g < tol_g, rel_g


@pytest.mark.parametrize("shape_s,shape_t", [((64, 256, 8, 8), (64, 256, 8, 8)),
                                             ((32, 64, 16, 16), (32, 128, 8, 8)),
                                             ((64, 256), (64, 128))])
def test_sp_native_matches_reference(shape_s, shape_t):
    f_s, f_t = _feat(shape_s, True, seed=1), _feat(shape_t, True, seed=2)
    assert FL._relation_native_ok(f_s, f_t)
    ln, lr, gn, gr = _run(FL.similarity_loss, FL.similarity_loss_ref, f_s, f_t)
    assert ln.shape == lr.shape == (1,)
    _check(ln, lr, gn, gr)


@pytest.mark.parametrize("shape_s,shape_t", [((64, 256), (64, 256)), ((48, 64), (48, 128)),
                                             ((64, 128, 4, 4), (64, 256, 4, 4))])
def test_pkt_native_matches_reference(shape_s, shape_t):
    f_s, f_t = _feat(shape_s, True, seed=3), _feat(shape_t, True, seed=4)
    ln, lr, gn, gr = _run(FL.pkt_loss, FL.pkt_loss_ref, f_s, f_t)
    _check(ln, lr, gn, gr)


@pytest.mark.parametrize("squared", [False, True])
@pytest.mark.parametrize("shape_s,shape_t", [((64, 256), (64, 256)), ((40, 64), (40, 128))])
def test_rkd_native_matches_reference(shape_s, shape_t, squared):
    f_s, f_t = _feat(shape_s, True, seed=5), _feat(shape_t, True, seed=6)

    def nat(a, b):
        return FL.rkd_loss(a, b, squared, 1e-12, 25.0, 50.0)

    def ref(a, b):
        return FL.rkd_loss_ref(a, b, squared, 1e-12, 25.0, 50.0)

    ln, lr, gn, gr = _run(nat, ref, f_s, f_t)
    _check(ln, lr, gn, gr)


def test_relation_takes_native_path_and_falls_back():
    f_s, f_t = _feat((64, 256), False), _feat((64, 256), False, seed=7)
    assert FL._relation_native_ok(f_s, f_t)
    assert not FL._relation_native_ok(_feat((65, 256), False), _feat((65, 256), False))
    assert any(p.endswith("libmda_hip.so") for p in _ext.LOADED_PATHS) or _ext.available()
    # > 64 rows: the PyTorch form runs
    big_s, big_t = _feat((80, 64), False), _feat((80, 64), False, seed=8)
    out = FL.rkd_loss(big_s.float(), big_t.float())
    assert torch.isfinite(out)


def test_rkd_graph_capture_replays():
    """The loss + backward launch sequence is capturable and replays with new inputs."""
    f_s = _feat((64, 256), False, seed=9).requires_grad_(True)
    f_t = _feat((64, 256), False, seed=10)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(2):
            f_s.grad = None
            FL.rkd_loss(f_s, f_t).backward()
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    f_s.grad = None
    with torch.cuda.graph(g):
        loss = FL.rkd_loss(f_s, f_t)
        loss.backward()
    with torch.no_grad():
        f_s.copy_(_feat((64, 256), False, seed=11))
    g.replay()
    torch.cuda.synchronize()
    b = f_s.detach().float().clone().requires_grad_(True)
    lr = FL.rkd_loss_ref(b, f_t.float())
    lr.backward()
    assert abs(loss.item() - lr.item()) / abs(lr.item()) < 2e-3
    assert ((f_s.grad.float() - b.grad).norm() / b.grad.norm()).item() < 2e-2
