"""KDSVD's SVD through the W x W Gram eigendecomposition (ops/feat_losses.py
_GramEig / _svd_gram) against torch.linalg.svd -- the reference's
distillers/KDSVD.py:8-25 -- on CPU in float64.  Singular vectors are defined
up to sign, so vectors are compared after fixing LAPACK's signs to the native
convention (largest-magnitude component positive), and gradients on
sign-invariant functions."""
import torch

from mdistiller_ddp_amd.ops import feat_losses as FL


def _fix_signs(v):
    idx = v.abs().argmax(dim=1, keepdim=True)
    return v * torch.where(v.gather(1, idx) < 0, -1.0, 1.0).to(v.dtype)


def test_gram_eig_gradcheck():
    torch.manual_seed(0)
    x = torch.randn(3, 12, 6, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(lambda t: FL._GramEig.apply(t), (x,))


def test_svd_gram_matches_svd():
    torch.manual_seed(1)
    f = torch.randn(4, 8, 6, 8, dtype=torch.float64)
    for n in (1, 4, 7):
        _, s_ref, v_ref = FL._svd(f, n)
        _, s, v = FL._svd_gram(f, n)  # both paths cast to fp32 as the reference does
        torch.testing.assert_close(s, s_ref, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(v, _fix_signs(v_ref), atol=1e-4, rtol=1e-4)


def test_svd_gram_gradient_matches_svd():
    torch.manual_seed(2)
    f0 = torch.randn(4, 8, 6, 8, dtype=torch.float64)
    w = torch.randn(4, 8, 5, dtype=torch.float64)

    def grad(fn):
        f = f0.clone().requires_grad_(True)
        _, _, v = fn(f, 5)
        ((v * v) * w).sum().backward()  # invariant to each column's sign
        return f.grad

    def svd64(f, n):  # the reference path without its fp32 cast
        N, C, H, W = f.shape
        _, _, vh = torch.linalg.svd(f.reshape(N, C * H, W), full_matrices=False)
        return None, None, torch.nn.functional.normalize(vh.transpose(-2, -1)[:, :, :n], dim=1)

    def gram64(f, n):
        N, C, H, W = f.shape
        _, v = FL._GramEig.apply(f.reshape(N, C * H, W))
        return None, None, torch.nn.functional.normalize(v[:, :, :n], dim=1)

    torch.testing.assert_close(grad(gram64), grad(svd64), atol=1e-8, rtol=1e-6)


def test_kdsvd_loss_native_matches_svd_path_with_same_signs(monkeypatch):
    """The whole loss: both paths agree once the rocSOLVER/LAPACK path uses
    the same sign convention."""
    torch.manual_seed(3)
    g_s = [torch.randn(4, c, h, h, dtype=torch.float64) for c, h in ((8, 8), (16, 4), (32, 2))]
    g_t = [torch.randn(4, c, h, h, dtype=torch.float64) for c, h in ((16, 8), (32, 4), (64, 2))]
    ref_svd = FL._svd

    def svd_fixed(feat, n=1):
        u, s, v = ref_svd(feat, n)
        return u, s, _fix_signs(v)

    g_s2 = [t.clone().requires_grad_(True) for t in g_s]
    g_s = [t.requires_grad_(True) for t in g_s]
    ln = FL.kdsvd_loss(g_s, g_t, 1, native=True)
    monkeypatch.setattr(FL, "_svd", svd_fixed)
    lr = FL.kdsvd_loss(g_s2, g_t, 1, native=False)
    torch.testing.assert_close(ln, lr, atol=1e-4, rtol=1e-4)
    # gradients too (the native path skips V's normalisation: an identity
    # whose backward only touches what the eigenvector gradient ignores)
    ln.backward()
    lr.backward()
    for a, b in zip(g_s, g_s2):
        assert (a.grad - b.grad).norm() <= 1e-3 * b.grad.norm()
