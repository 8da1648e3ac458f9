"""KDSVD's native Jacobi eigensolver (csrc/eig.hip mda_sym_eig) against
torch.linalg.eigh in float64 with the same order / sign convention, the loss
and its gradient against the CPU path, and the loss captured in a hipGraph
(rocSOLVER's SVD could not be)."""
import pytest
import torch

from mdistiller_ddp_amd.ops import _ext
from mdistiller_ddp_amd.ops import feat_losses as FL

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, scope="module")
def _native():
    _ext.load(required=True)


@pytest.mark.parametrize("n", [2, 7, 8, 16, 32, 63])
def test_sym_eig_matches_eigh(n):
    torch.manual_seed(n)
    x = torch.randn(16, 3 * n, n, dtype=torch.float64)
    g = x.transpose(1, 2) @ x
    lam_ref, v_ref = FL._GramEig.apply(x)  # CPU: eigh, same convention
    lam = torch.empty(16, n, device="cuda")
    v = torch.empty(16, n, n, device="cuda")
    _ext.call("mda_sym_eig", g.float().cuda().contiguous(), 16, n, 8, lam, v)
    torch.cuda.synchronize()
    torch.testing.assert_close(lam.cpu().double(), lam_ref, rtol=1e-5, atol=1e-4 * lam_ref.abs().max().item())
    torch.testing.assert_close(v.cpu().double(), v_ref, atol=2e-4, rtol=0)


def _feats(seed, dev):
    torch.manual_seed(seed)
    g_s = [torch.randn(64, c, h, h) for c, h in ((32, 32), (64, 16), (128, 8))]
    g_t = [torch.randn(64, c, h, h) for c, h in ((64, 32), (128, 16), (256, 8))]
    return [t.to(dev).requires_grad_(True) for t in g_s], [t.to(dev) for t in g_t]


def test_kdsvd_loss_gpu_matches_cpu():
    gs_c, gt_c = _feats(0, "cpu")
    gs_g, gt_g = _feats(0, "cuda")
    assert FL.kdsvd_native_ok(gs_g, gt_g)
    lc = FL.kdsvd_loss(gs_c, gt_c, 1)
    lg = FL.kdsvd_loss(gs_g, gt_g, 1)
    lc.backward()
    lg.backward()
    torch.testing.assert_close(lg.cpu(), lc, rtol=1e-3, atol=1e-4)
    for a, b in zip(gs_g, gs_c):
        rel = (a.grad.cpu() - b.grad).norm() / b.grad.norm().clamp_min(1e-30)
        assert rel < 1e-2


def test_kdsvd_loss_graph_capture_matches_eager():
    g_s, g_t = _feats(1, "cuda")
    static_s = [t.detach().clone().requires_grad_(True) for t in g_s]
    eager = FL.kdsvd_loss(static_s, g_t, 1)
    eager.backward()
    ref_grads = [t.grad.clone() for t in static_s]
    for t in static_s:
        t.grad = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):  # warm-up on the capture stream
            FL.kdsvd_loss(static_s, g_t, 1).backward()
            for t in static_s:
                t.grad = None
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = FL.kdsvd_loss(static_s, g_t, 1)
        out.backward()
    graph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, eager, rtol=1e-5, atol=1e-6)
    for t, r in zip(static_s, ref_grads):
        torch.testing.assert_close(t.grad, r, rtol=1e-4, atol=1e-6)
