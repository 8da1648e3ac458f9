"""Native NHWC max pooling (csrc/pool.hip) vs PyTorch fp32, and the
channel-padded stem input (csrc/conv_wgrad.hip::pad_channels)."""
import pytest
import torch
import torch.nn.functional as F

from mdistiller_ddp_amd.ops import nn as mnn
from mdistiller_ddp_amd.ops import hip_train
from mdistiller_ddp_amd.ops.backend import use_backend

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,C,H,k,s,p", [(4, 64, 112, 3, 2, 1), (8, 64, 32, 2, 2, 0),
                                         (3, 16, 15, 3, 2, 1), (2, 256, 8, 2, 2, 0),
                                         (2, 8, 9, 3, 1, 1)])
def test_maxpool_fwd_bwd(N, C, H, k, s, p):
    torch.manual_seed(0)
    # distinct values: no ties, so the argmax (and gradient) is unambiguous
    x = torch.randperm(N * C * H * H, device="cuda").float().reshape(N, C, H, H) / (N * C * H * H)
    x = x.to(torch.bfloat16)
    x = x + 0 * x  # keep bf16
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    xh = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    with use_backend("hip"):
        y = mnn.max_pool2d(xh, k, s, p)
    assert y.is_contiguous(memory_format=torch.channels_last)
    y.backward(g.to(torch.bfloat16))
    torch.testing.assert_close(y.float(), yr.detach(), atol=0, rtol=0)
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pad_channels8(dtype):
    x = torch.randn(3, 3, 17, 19, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    y = hip_train.pad_channels8(x)
    assert y.shape == (3, 8, 17, 19) and y.dtype == torch.bfloat16
    torch.testing.assert_close(y[:, :3].float(), x.to(torch.bfloat16).float(), atol=0, rtol=0)
    assert torch.count_nonzero(y[:, 3:]) == 0
    assert hip_train.pad_channels8(x) is y  # cached for the same version / stream
    x.add_(1.0)
    assert hip_train.pad_channels8(x) is not y


@pytest.mark.parametrize("C,g", [(240, 3), (58, 2), (120, 4)])
def test_channel_shuffle_native(C, g):
    from mdistiller_ddp_amd.ops import nn as mnn
    from mdistiller_ddp_amd.ops.backend import use_backend
    torch.manual_seed(0)
    x = torch.randn(4, C, 6, 5, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xh = x.clone().requires_grad_(True)
    with use_backend("hip"):
        y = mnn.channel_shuffle(xh, g)
    n, c, h, w = x.shape
    ref = x.float().reshape(n, g, c // g, h, w).transpose(1, 2).reshape(n, c, h, w)
    torch.testing.assert_close(y.float(), ref, rtol=0, atol=0)
    go = torch.randn_like(ref)
    y.backward(go.to(torch.bfloat16))
    xr = x.float().clone().requires_grad_(True)
    (xr.reshape(n, g, c // g, h, w).transpose(1, 2).reshape(n, c, h, w) * go.to(torch.bfloat16).float()).sum().backward()
    torch.testing.assert_close(xh.grad.float(), xr.grad, rtol=0, atol=0)


@pytest.mark.parametrize("N,C3,Cx,H", [(8, 216, 24, 32), (4, 240, 240, 16), (3, 480, 480, 8), (2, 16, 8, 7)])
def test_shuffle_tail_matches_torch(N, C3, Cx, H):
    """ShuffleNetV1 stride-2 tail (csrc/pool.hip mda_shuffle_tail_*): cat with
    the 3x3/s2 average-pooled shortcut + ReLU, and its backward, vs PyTorch fp32."""
    import torch.nn.functional as F
    from mdistiller_ddp_amd.ops.nn import shuffle_tail
    torch.manual_seed(0)
    Ho = (H + 1) // 2
    y3 = torch.randn(N, C3, Ho, Ho, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = torch.randn(N, Cx, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a, b = y3.clone().requires_grad_(True), x.clone().requires_grad_(True)
    out, pre = shuffle_tail(a, b)
    # fp32 reference on the CPU, NCHW: this ROCm build's channels_last
    # avg_pool2d backward on the GPU shifts the gradient by one column (its
    # single-output border column lands at w = 0 instead of w = W - 1)
    ar = y3.float().cpu().contiguous().requires_grad_(True)
    br = x.float().cpu().contiguous().requires_grad_(True)
    pre_r = torch.cat([ar, F.avg_pool2d(br, 3, stride=2, padding=1)], 1)
    out_r = F.relu(pre_r)
    rel = lambda u, v: ((u.float().cpu() - v.float()).norm() / v.float().norm()).item()  # noqa: E731
    assert rel(pre, pre_r) < 1e-2 and rel(out, out_r) < 1e-2
    g, gp = torch.randn_like(out_r), torch.randn_like(out_r)
    ((out.float() * g.cuda()).sum() + (pre.float() * gp.cuda()).sum()).backward()
    ((out_r * g).sum() + (pre_r * gp).sum()).backward()
    assert rel(a.grad, ar.grad) < 1e-2
    assert rel(b.grad, br.grad) < 1e-2
