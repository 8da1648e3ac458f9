"""Feature / relation distillation losses.

Formulas follow the reference distillers line by line (cited per function);
the implementations are written for the device: fp32 math on bf16
activations, Gram-form kernels instead of materialised B x B x D tensors
where the algebra allows, the AT loss as a fused HIP kernel
(``csrc/feat.hip``) and SP / PKT / RKD on the batch Gram
(``csrc/relation.hip``) on MI355X; ``*_ref`` are the PyTorch forms (CPU and
unsupported shapes).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext
from .backend import hip_enabled_for


def _pool_to_match(f_s, f_t):
    s_H, t_H = f_s.shape[2], f_t.shape[2]
    if s_H > t_H:
        f_s = F.adaptive_avg_pool2d(f_s, (t_H, t_H))
    elif s_H < t_H:
        f_t = F.adaptive_avg_pool2d(f_t, (s_H, s_H))
    return f_s, f_t


# ---------------------------------------------------------------- AT (K8)
def _at_map(feat, p):
    return F.normalize(feat.float().pow(p).mean(1).reshape(feat.size(0), -1))


def single_stage_at_loss_ref(f_s, f_t, p):
    """`distillers/AT.py:8-18`."""
    f_s, f_t = _pool_to_match(f_s, f_t)
    return (_at_map(f_s, p) - _at_map(f_t, p)).pow(2).mean()


class _ATLoss(torch.autograd.Function):
    """Fused: a = mean_c f^p per pixel -> L2-normalise over HW -> mean sq diff.

    Teacher map is constant; the kernel writes the loss and d loss / d f_s.
    """

    @staticmethod
    def forward(ctx, f_s, f_t, p):
        f_s = f_s.contiguous(memory_format=torch.channels_last)
        f_t = f_t.contiguous(memory_format=torch.channels_last)
        N, C, H, W = f_s.shape
        Ct = f_t.shape[1]
        grad = torch.empty_like(f_s)
        loss = torch.empty(1, dtype=torch.float32, device=f_s.device)
        dt_s = 1 if f_s.dtype == torch.bfloat16 else 0
        dt_t = 1 if f_t.dtype == torch.bfloat16 else 0
        from .losses import workspace
        ws = workspace(f_s.device)
        _ext.call("mda_at_loss", dt_s, dt_t, f_s, f_t, grad, loss, ws.partial, ws.counter, N, C, Ct,
                  H * W, float(p))
        ctx.save_for_backward(grad)
        return loss[0]

    @staticmethod
    def backward(ctx, go):
        grad, = ctx.saved_tensors
        return grad * go.to(grad.dtype), None, None


def single_stage_at_loss(f_s, f_t, p):
    f_s, f_t = _pool_to_match(f_s, f_t)
    if (hip_enabled_for(f_s) and f_s.dim() == 4 and f_s.shape[2:] == f_t.shape[2:]
            and f_s.dtype in (torch.float32, torch.bfloat16) and f_t.dtype in (torch.float32, torch.bfloat16)
            and f_s.shape[2] * f_s.shape[3] <= 4096 and float(p) == 2.0):
        return _ATLoss.apply(f_s, f_t.detach(), p)
    return single_stage_at_loss_ref(f_s, f_t, p)


def at_loss(g_s, g_t, p):
    return sum(single_stage_at_loss(f_s, f_t, p) for f_s, f_t in zip(g_s, g_t))


# ---------------------------------------------------------------- NST
def single_stage_nst_loss(f_s, f_t):
    """`distillers/NST.py:12-35`: polynomial (a.b)^2 kernel MMD.

    mean_{ij} (f_i . g_j)^2 over channel pairs = ||F G^T||_F^2 / C_f C_g,
    computed as batched Gram products (MFMA GEMMs) instead of broadcasting
    an (N, C, C, HW) tensor.
    """
    f_s, f_t = _pool_to_match(f_s, f_t)

    def rows(f):
        # [N, HW, C] channel columns: a free view of a channels_last map (the
        # [N, C, HW] view of one costs a transposing copy, fwd and bwd)
        n, c = f.shape[0], f.shape[1]
        if f.is_contiguous(memory_format=torch.channels_last) and not f.is_contiguous():
            return f.permute(0, 2, 3, 1).reshape(n, -1, c).float()
        return f.float().reshape(n, c, -1).transpose(1, 2)

    f_s = F.normalize(rows(f_s), dim=1)
    f_t = F.normalize(rows(f_t), dim=1)

    def kmean(a, b):  # mean_{cd} (a_c . b_d)^2 with a, b [N, HW, C]
        return torch.bmm(a.transpose(1, 2), b).pow(2).mean()

    return kmean(f_t, f_t).detach() + kmean(f_s, f_s) - 2 * kmean(f_s, f_t)


class _NSTGram(torch.autograd.Function):
    """NST on ONE Gram per sample: with W = [F_s | F_t] ([HW, 2C] channel
    columns), G = W^T W holds all three raw Grams; F.normalize's column norms
    are sqrt(diag G), so the normalised Grams are G / (r_i r_j) and the loss
    is (||S||^2 + ||T||^2 - 2||X||^2) / (N C^2) -- no pass over the feature
    maps besides the one batched GEMM.  Backward in closed form:
        dot_c = k (sum_d S_cd^2 - sum_d X_cd^2),  k = 4 go / (N C^2)
        P = D_s (k S - diag(dot)) D_s,  Q = -k D_t X^T D_s,   D = diag(1/r)
        dF_s = F_s P + F_t Q = W [P; Q]          (one batched GEMM)
    On the GPU the Gram algebra runs in csrc/feat.hip (mda_nst_fwd /
    mda_nst_bwd); elsewhere in PyTorch ops.
    """

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, fs_cols, ft_cols):
        # [N, HW, C] each; fp32 GEMMs (autocast off)
        w = torch.cat([fs_cols, ft_cols], 2).float()
        N, _, C2 = w.shape
        C = C2 // 2
        g = torch.bmm(w.transpose(1, 2), w)
        native = g.is_cuda and hip_enabled_for(g) and C <= 1024
        if native:
            part = torch.empty(N, (C2 + 31) // 32, dtype=torch.float32, device=g.device)
            _ext.call("mda_nst_fwd", g, N, C, part)
            loss = part.sum() / (N * C * C)
        else:
            r = g.diagonal(dim1=1, dim2=2).clamp_min(0).sqrt().clamp_min(1e-12)
            gh = g / (r.unsqueeze(2) * r.unsqueeze(1))
            S, X, T = gh[:, :C, :C], gh[:, :C, C:], gh[:, C:, C:]
            loss = (S.square().sum() + T.square().sum() - 2 * X.square().sum()) / (N * C * C)
        ctx.save_for_backward(w, g)
        ctx.native = native
        return loss

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, go):
        w, g = ctx.saved_tensors
        N, _, C2 = w.shape
        C = C2 // 2
        if ctx.native:
            pq = torch.empty(N, C2, C, dtype=torch.float32, device=g.device)
            _ext.call("mda_nst_bwd", g, N, C, go.detach().float().reshape(1).contiguous(), pq)
        else:
            r = g.diagonal(dim1=1, dim2=2).clamp_min(0).sqrt().clamp_min(1e-12)
            gh = g / (r.unsqueeze(2) * r.unsqueeze(1))
            S, X = gh[:, :C, :C], gh[:, :C, C:]
            k = 4.0 * go / (N * C * C)
            rs, rt = r[:, :C], r[:, C:]
            dot = k * (S.square().sum(2) - X.square().sum(2))
            P = (k * S - torch.diag_embed(dot)) / (rs.unsqueeze(2) * rs.unsqueeze(1))
            Q = -k * X.transpose(1, 2) / (rt.unsqueeze(2) * rs.unsqueeze(1))
            pq = torch.cat([P, Q], 1)
        return torch.bmm(w, pq), None


def _nst_cols(f):
    """[N, HW, C] channel columns: a free view of a channels_last map."""
    n, c = f.shape[0], f.shape[1]
    if f.is_contiguous(memory_format=torch.channels_last) and not f.is_contiguous():
        return f.permute(0, 2, 3, 1).reshape(n, -1, c)
    return f.reshape(n, c, -1).transpose(1, 2)


def single_stage_nst_loss_gram(f_s, f_t):
    """:func:`single_stage_nst_loss` through :class:`_NSTGram` (one batched
    Gram forward, one batched product backward)."""
    f_s, f_t = _pool_to_match(f_s, f_t.detach())
    if f_s.shape[1] != f_t.shape[1]:
        return single_stage_nst_loss(f_s, f_t)
    return _NSTGram.apply(_nst_cols(f_s), _nst_cols(f_t))


def nst_loss(g_s, g_t):
    if g_s and hip_enabled_for(g_s[0]):
        return sum(single_stage_nst_loss_gram(f_s, f_t) for f_s, f_t in zip(g_s, g_t))
    return sum(single_stage_nst_loss(f_s, f_t) for f_s, f_t in zip(g_s, g_t))


# ------------------------------------------------- native Gram-form relations
# SP, PKT and RKD on the batch Gram G = F F^T (csrc/relation.hip): one MFMA
# Gram launch over the features, the B x B algebra and its gradient dL/dG in
# one (SP/PKT) or two (RKD) launches, and dF = go (dG + dG^T) F in the backward.
_REL_SP, _REL_PKT, _REL_RKD = 0, 1, 2


def _flat_bf16(f):
    """[B, D] bf16 row-major view of ``f`` in its memory order (see :func:`_flat`)."""
    n = f.shape[0]
    if f.dim() == 4 and f.is_contiguous(memory_format=torch.channels_last) and not f.is_contiguous():
        v = f.permute(0, 2, 3, 1).reshape(n, -1)
    else:
        v = f.reshape(n, -1)
    if v.dtype != torch.bfloat16:
        v = v.to(torch.bfloat16)
    return v.contiguous()


def _gram_plan(D):
    import ctypes
    kc, nc = ctypes.c_int64(0), ctypes.c_int64(0)
    _ext.call("mda_gram_plan", D, kc, nc)
    return kc.value, nc.value


class _RelationLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f_s, f_t, mode, squared, eps, dist_w, angle_w):
        a_s, a_t = _flat_bf16(f_s), _flat_bf16(f_t)
        B, Ds = a_s.shape
        Dt = a_t.shape[1]
        kc_s, nc_s = _gram_plan(Ds)
        kc_t, nc_t = _gram_plan(Dt)
        dev = a_s.device
        part = torch.empty((nc_s + nc_t) * 4096, dtype=torch.float32, device=dev)
        _ext.call("mda_gram_partial", a_s, a_t, part, B, Ds, Dt, kc_s, kc_t, nc_s, nc_t)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        S = torch.empty(64 * 64, dtype=torch.float32, device=dev)
        if mode == _REL_RKD:
            scratch = torch.empty(3 * 4096 + 64, dtype=torch.float32, device=dev)
            _ext.call("mda_rkd_loss", part, nc_s, nc_t, B, int(bool(squared)), float(eps),
                      float(dist_w), float(angle_w), scratch[:4096], scratch[4096:8192],
                      scratch[8192:12288], scratch[12288:], loss, S)
        else:
            _ext.call("mda_relation_core", part, nc_s, nc_t, B, mode, loss, S)
        ctx.save_for_backward(a_s, S)
        ctx.fshape = (f_s.shape, f_s.dtype, f_s.dim() == 4 and not f_s.is_contiguous()
                      and f_s.is_contiguous(memory_format=torch.channels_last))
        return loss if mode == _REL_SP else loss[0]

    @staticmethod
    def backward(ctx, go):
        a_s, S = ctx.saved_tensors
        shape, dtype, cl = ctx.fshape
        B, D = a_s.shape
        g = torch.empty(shape, dtype=torch.bfloat16, device=a_s.device,
                        memory_format=torch.channels_last if cl else torch.contiguous_format)
        gflat = g.permute(0, 2, 3, 1).reshape(B, -1) if cl else g.reshape(B, -1)
        _ext.call("mda_gram_bwd", a_s, S, go.float().contiguous(), gflat, B, D)
        if dtype != torch.bfloat16:
            g = g.to(dtype)
        return g, None, None, None, None, None, None


def _relation_native_ok(f_s, f_t, min_batch=1) -> bool:
    if not hip_enabled_for(f_s):
        return False
    B = f_s.shape[0]
    if f_t.shape[0] != B or not (min_batch <= B <= 64):
        return False
    if f_s.dtype not in (torch.float32, torch.bfloat16) or f_t.dtype not in (torch.float32, torch.bfloat16):
        return False
    ds, dt = f_s[0].numel(), f_t[0].numel()
    return ds % 8 == 0 and dt % 8 == 0 and ds > 0 and dt > 0


# ---------------------------------------------------------------- PKT
def _flat(f):
    """``f.reshape(N, -1)`` in fp32 up to a fixed column permutation.

    PKT, SP and RKD only use row norms, row dot products and row differences, which
    are invariant to permuting the flattened columns, so a channels_last map is
    flattened in its memory order (a free view) instead of being made NCHW first.
    """
    n = f.shape[0]
    if f.dim() == 4 and f.is_contiguous(memory_format=torch.channels_last) and not f.is_contiguous():
        return f.permute(0, 2, 3, 1).reshape(n, -1).float()
    return f.float().reshape(n, -1)


def pkt_loss(f_s, f_t, eps=1e-7):
    """`distillers/PKT.py:8-35`."""
    if eps == 1e-7 and _relation_native_ok(f_s, f_t):
        return _RelationLoss.apply(f_s, f_t.detach(), _REL_PKT, False, 0.0, 0.0, 0.0)
    return pkt_loss_ref(f_s, f_t, eps)


def pkt_loss_ref(f_s, f_t, eps=1e-7):
    f_s = _flat(f_s)
    f_t = _flat(f_t)
    f_s = f_s / (f_s.pow(2).sum(1, keepdim=True).sqrt() + eps)
    f_s = torch.nan_to_num(f_s, nan=0.0)
    f_t = f_t / (f_t.pow(2).sum(1, keepdim=True).sqrt() + eps)
    f_t = torch.nan_to_num(f_t, nan=0.0)
    ms = (f_s @ f_s.t() + 1.0) / 2.0
    ts = (f_t @ f_t.t() + 1.0) / 2.0
    ms = ms / ms.sum(1, keepdim=True)
    ts = ts / ts.sum(1, keepdim=True)
    return torch.mean(ts * torch.log((ts + eps) / (ms + eps)))


# ---------------------------------------------------------------- SP
def similarity_loss(f_s, f_t):
    """`distillers/SP.py:12-24`."""
    if _relation_native_ok(f_s, f_t):
        return _RelationLoss.apply(f_s, f_t.detach(), _REL_SP, False, 0.0, 0.0, 0.0)
    return similarity_loss_ref(f_s, f_t)


def similarity_loss_ref(f_s, f_t):
    bsz = f_s.shape[0]
    f_s = _flat(f_s)
    f_t = _flat(f_t)
    G_s = F.normalize(f_s @ f_s.t())
    G_t = F.normalize(f_t @ f_t.t())
    d = G_t - G_s
    return (d * d).sum().reshape(1) / (bsz * bsz)


def sp_loss(g_s, g_t):
    return sum(similarity_loss(f_s, f_t) for f_s, f_t in zip(g_s, g_t))


# ---------------------------------------------------------------- RKD
def _pdist(e, squared, eps):
    e_sq = e.pow(2).sum(dim=1)
    prod = e @ e.t()
    res = (e_sq.unsqueeze(1) + e_sq.unsqueeze(0) - 2 * prod).clamp(min=eps)
    if not squared:
        res = res.sqrt()
    n = len(e)
    return res * (1.0 - torch.eye(n, device=e.device, dtype=res.dtype))


def _angles(x):
    """cos of the angle at i between (j - i) and (k - i), flattened (B^3)."""
    d = x.unsqueeze(0) - x.unsqueeze(1)
    d = F.normalize(d, p=2, dim=2)
    return torch.bmm(d, d.transpose(1, 2)).reshape(-1)


def _positive_mean(x):
    """``x[x > 0].mean()`` without a data-dependent shape (capture-safe)."""
    pos = (x > 0).to(x.dtype)
    return (x * pos).sum() / pos.sum()


def rkd_loss(f_s, f_t, squared=False, eps=1e-12, distance_weight=25, angle_weight=50):
    """`distillers/RKD.py:21-50`."""
    if _relation_native_ok(f_s, f_t, min_batch=2):
        return _RelationLoss.apply(f_s, f_t.detach(), _REL_RKD, squared, eps, distance_weight,
                                   angle_weight)
    return rkd_loss_ref(f_s, f_t, squared, eps, distance_weight, angle_weight)


def rkd_loss_ref(f_s, f_t, squared=False, eps=1e-12, distance_weight=25, angle_weight=50):
    stu = _flat(f_s)
    tea = _flat(f_t)
    with torch.no_grad():
        t_d = _pdist(tea, squared, eps)
        t_d = t_d / _positive_mean(t_d)
    d = _pdist(stu, squared, eps)
    d = d / _positive_mean(d)
    loss_d = F.smooth_l1_loss(d, t_d)
    with torch.no_grad():
        t_angle = _angles(tea)
    s_angle = _angles(stu)
    loss_a = F.smooth_l1_loss(s_angle, t_angle)
    return distance_weight * loss_d + angle_weight * loss_a


# ---------------------------------------------------------------- KDSVD
def _removenan(x):
    return torch.where(torch.isfinite(x), x, torch.zeros_like(x))


def _svd(feat, n=1):
    N, C, H, W = feat.shape
    # reference: view(N, C*H, W) of an NCHW tensor
    x = feat.float().contiguous().reshape(N, C * H, W)
    u, s, vh = torch.linalg.svd(x, full_matrices=False)
    v = vh.transpose(-2, -1)
    u, s, v = _removenan(u), _removenan(s), _removenan(v)
    if n > 0:
        u = F.normalize(u[:, :, :n], dim=1)
        s = F.normalize(s[:, :n], dim=1)
        v = F.normalize(v[:, :, :n], dim=1)
    return u, s, v


def _sym_eig(g):
    """(descending eigenvalues, eigenvector columns with their largest-magnitude
    component positive) of a batch of symmetric matrices; no autograd."""
    B, W, _ = g.shape
    if g.is_cuda:
        lam = torch.empty(B, W, dtype=torch.float32, device=g.device)
        vec = torch.empty(B, W, W, dtype=torch.float32, device=g.device)
        _ext.call("mda_sym_eig", g.float().contiguous(), B, W, 8, lam, vec)
        return lam, vec
    lam, vec = torch.linalg.eigh(g.double())
    lam, vec = lam.flip(-1), vec.flip(-1)
    idx = vec.abs().argmax(dim=1, keepdim=True)
    vec = vec * torch.where(vec.gather(1, idx) < 0, -1.0, 1.0)
    return lam.to(g.dtype), vec.to(g.dtype)


_EIG_DEGEN = 1e-6


class _GramEig(torch.autograd.Function):
    """Eigenvalues (descending) and eigenvectors (columns; largest-magnitude
    component positive) of G = X^T X for a batch X [B, R, W], W <= 63: the
    squared singular values and right singular vectors of X.  ``x_other``
    (optional, [B', R', W], no gradient): another batch whose Grams are
    diagonalised in the same launch (KDSVD's teacher stage), returned second.

    GPU: the Gram on rocBLAS, the eigensolver on the native Jacobi kernel
    (csrc/eig.hip) -- nothing synchronises with the host, so KDSVD captures
    into the step graph.  CPU: torch.linalg.eigh with the same order and sign
    convention.  Backward (either way): with K = F o (V^T dV),
    F_ij = 1 / (lam_j - lam_i) off the diagonal, dG = V (K + diag(dlam)) V^T
    and dX = X (dG + dG^T) -- the SVD's V / sigma^2 gradient for distinct
    singular values."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, x_other=None):
        B = x.shape[0]
        g = torch.bmm(x.transpose(1, 2), x)
        if x_other is not None:
            g = torch.cat([g, torch.bmm(x_other.transpose(1, 2), x_other)])
        lam, vec = _sym_eig(g.contiguous())
        lam_s, vec_s = lam[:B], vec[:B]
        ctx.save_for_backward(x, lam_s, vec_s)
        if x_other is None:
            return lam_s, vec_s
        lam_o, vec_o = lam[B:], vec[B:]
        ctx.mark_non_differentiable(lam_o, vec_o)
        return lam_s, vec_s, lam_o, vec_o

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dlam, dvec, *unused):
        x, lam, v = ctx.saved_tensors
        k = torch.zeros_like(v)
        if dvec is not None:
            diff = lam.unsqueeze(1) - lam.unsqueeze(2)  # [i, j] = lam_j - lam_i
            # gaps below 1e-6 of the largest eigenvalue (the fp32 solver's
            # resolution) are one degenerate subspace: no 1/gap term (the SVD
            # backward's 1/(s_j^2 - s_i^2) otherwise amplifies rounding noise
            # by orders of magnitude; csrc/kdsvd.hip KS_DEGEN)
            thr = _EIG_DEGEN * lam.abs().amax(dim=1, keepdim=True).unsqueeze(2)
            f = torch.where(diff.abs() > thr, 1.0 / diff, torch.zeros_like(diff))
            f.diagonal(dim1=1, dim2=2).zero_()
            k = f * torch.bmm(v.transpose(1, 2), dvec)
        if dlam is not None:
            k = k + torch.diag_embed(dlam)
        dg = torch.bmm(torch.bmm(v, k), v.transpose(1, 2))
        return torch.bmm(x, dg + dg.transpose(1, 2)), None


def _svd_native_ok(feat) -> bool:
    N, C, H, W = feat.shape
    if not (2 <= W <= 63 and C * H >= W and N <= 65535):
        return False
    return not feat.is_cuda or _ext.available()


def _svd_gram(feat, n=1):
    """``_svd`` through the Gram eigendecomposition (no U: KDSVD never uses
    it); same normalisation of the leading n singular values / vectors."""
    N, C, H, W = feat.shape
    x = feat.float().contiguous().reshape(N, C * H, W)
    lam, v = _GramEig.apply(x)
    return _svd_post(lam, v, n)


def _svd_post(lam, v, n, exact=False):
    """``exact``: v came from the eigensolver, finite with unit columns -- the
    reference's NaN scrub and column normalisation of V are then identities
    (and so is normalize's backward: it only removes dV's component along
    each v_j, which the eigenvector gradient ignores), so they are skipped."""
    s = lam.clamp_min(0).sqrt()
    if not exact:
        s, v = _removenan(s), _removenan(v)
    if n > 0:
        s = F.normalize(s[:, :n], dim=1)
        v = v[:, :, :n] if exact else F.normalize(v[:, :, :n], dim=1)
    return None, s, v


def _align_rsv(a, b):
    cosine = torch.matmul(a.transpose(-2, -1), b)
    max_abs, _ = torch.max(torch.abs(cosine), 1, keepdim=True)
    mask = torch.where(torch.eq(max_abs, torch.abs(cosine)), torch.sign(cosine),
                       torch.zeros_like(cosine))
    return torch.matmul(a, mask), b


class _KdsvdPost(torch.autograd.Function):
    """The KDSVD loss from the stages' eigendecompositions (csrc/kdsvd.hip):
    sign alignment of the k+3 leading student vectors to the k teacher ones,
    teacher-singular-value scaling, inter-stage RBF and L2 -- one launch
    forward, one backward (the PyTorch composition of :func:`kdsvd_loss`'s
    fallback is ~450 elementwise kernels per step).  Inputs: k, the teacher
    eigenvalue / eigenvector lists (no gradient), then the student
    eigenvector batches [N, W, W] (columns)."""

    @staticmethod
    def forward(ctx, k, lt, vt, *vs):
        S, N = len(vs), vs[0].shape[0]
        vs = [v.contiguous() for v in vs]
        vt = [v.contiguous() for v in vt]
        lt = [v.contiguous() for v in lt]
        W = [v.shape[-1] for v in vs]
        part = torch.empty(N, dtype=torch.float32, device=vs[0].device)
        tab = _kdsvd_table(vs, vt, lt, None, W)
        _ext.call("mda_kdsvd_post", *tab, S, N, k, part, None, None, None)
        ctx.save_for_backward(*vs, *vt, *lt)
        ctx.meta = (k, S, N, W)
        return part.sum()

    @staticmethod
    def backward(ctx, go):
        k, S, N, W = ctx.meta
        t = ctx.saved_tensors
        vs, vt, lt = list(t[:S]), list(t[S:2 * S]), list(t[2 * S:])
        dvs = [torch.empty_like(v) for v in vs]
        tab = _kdsvd_table(vs, vt, lt, dvs, W)
        _ext.call("mda_kdsvd_post", *tab, S, N, k, None, go.float().reshape(1).contiguous(), None, None)
        return (None, None, None) + tuple(dvs)


_KDSVD_KSPLIT = 4  # row ranges per sample in the Gram launch (partials summed by the eigensolver)


def _nhwc(f):
    return f.contiguous(memory_format=torch.channels_last)


class _KdsvdNative(torch.autograd.Function):
    """The whole KDSVD loss on the native kernels, from the NHWC feature maps:
    forward = ONE Gram launch for every stage's student and teacher
    (csrc/kdsvd.hip mda_kdsvd_gram, bf16/fp32 in, fp32 split-K partials) +
    ONE eigensolver launch for all stages (csrc/eig.hip mda_sym_eig_multi) +
    the post-processing launch; backward = the post-processing launch in D
    mode (through the eigendecomposition's backward: D = dG + dG^T) + ONE
    dX = X D launch for every stage.  Same algebra as the composition
    _GramEig + _KdsvdPost (which the tests pin it against); ~6 launches per
    step instead of ~100 (profiles/r4_prof_kdsvd.md)."""

    @staticmethod
    def forward(ctx, k, S, *feats):
        fs = [_nhwc(f.detach()) for f in feats[:S]]
        ft = [_nhwc(f.detach()) for f in feats[S:]]
        N, dev, ks = fs[0].shape[0], fs[0].device, _KDSVD_KSPLIT
        grams, rows = [], []
        for a, b in zip(fs, ft):
            W = a.shape[3]
            gp = torch.empty(ks, 2 * N, W, W, dtype=torch.float32, device=dev)
            grams.append(gp)
            for side, x in ((0, a), (1, b)):
                _, C, H, _ = x.shape
                rows.append([x.data_ptr(), gp.data_ptr() + side * N * W * W * 4, 2 * N * W * W,
                             N, H, W, C, int(x.dtype == torch.bfloat16)])
        _ext.call("mda_kdsvd_gram", torch.tensor(rows, dtype=torch.int64), len(rows), ks)
        lams, vecs, erows = [], [], []
        for gp in grams:
            W = gp.shape[-1]
            lam = torch.empty(2 * N, W, dtype=torch.float32, device=dev)
            vec = torch.empty(2 * N, W, W, dtype=torch.float32, device=dev)
            lams.append(lam)
            vecs.append(vec)
            erows.append([gp.data_ptr(), lam.data_ptr(), vec.data_ptr(), 2 * N * W * W, 2 * N, W, ks])
        _ext.call("mda_sym_eig_multi", torch.tensor(erows, dtype=torch.int64), len(erows), 8)
        Ws = [v.shape[-1] for v in vecs]
        part = torch.empty(N, dtype=torch.float32, device=dev)
        tab = _kdsvd_table([v[:N] for v in vecs], [v[N:] for v in vecs], [l[N:] for l in lams], None, Ws)
        _ext.call("mda_kdsvd_post", *tab, S, N, k, part, None, None, None)
        ctx.save_for_backward(*fs, *lams, *vecs)
        ctx.meta = (k, S, N, Ws)
        return part.sum()

    @staticmethod
    def backward(ctx, go):
        k, S, N, Ws = ctx.meta
        t = ctx.saved_tensors
        fs, lams, vecs = t[:S], t[S:2 * S], t[2 * S:]
        dev = fs[0].device
        ds = [torch.empty(N, W, W, dtype=torch.float32, device=dev) for W in Ws]
        tab = _kdsvd_table([v[:N] for v in vecs], [v[N:] for v in vecs], [l[N:] for l in lams], None, Ws)
        ls = torch.tensor([l.data_ptr() for l in lams], dtype=torch.int64)  # student rows first
        dptr = torch.tensor([d.data_ptr() for d in ds], dtype=torch.int64)
        _ext.call("mda_kdsvd_post", *tab, S, N, k, None, go.detach().float().reshape(1).contiguous(),
                  ls, dptr)
        dx = [torch.empty_like(f) for f in fs]
        rows = [[f.data_ptr(), d.data_ptr(), g.data_ptr(), N, f.shape[2], f.shape[3], f.shape[1],
                 int(f.dtype == torch.bfloat16)] for f, d, g in zip(fs, ds, dx)]
        _ext.call("mda_kdsvd_gram_apply", torch.tensor(rows, dtype=torch.int64), S)
        return (None, None) + tuple(dx) + (None,) * S


def kdsvd_native_full_ok(g_s, g_t, k) -> bool:
    """:class:`_KdsvdNative` serves (on top of :func:`kdsvd_fused_ok`): bf16 /
    fp32 feature maps, one batch size."""
    return (kdsvd_fused_ok(g_s, g_t, k)
            and all(f.dtype in (torch.bfloat16, torch.float32) and f.dim() == 4
                    and f.shape[0] == g_s[0].shape[0] for f in list(g_s) + list(g_t)))


def _kdsvd_table(vs, vt, lt, dvs, W):
    """Host pointer arrays of :func:`mda_kdsvd_post` (kept alive by the caller's frame)."""
    def arr(ts):
        return torch.tensor([t.data_ptr() if t is not None else 0 for t in ts], dtype=torch.int64)
    return (arr(vs), arr(vt), arr(lt), arr(dvs if dvs is not None else [None] * len(vs)),
            torch.tensor(W, dtype=torch.int64))


def kdsvd_fused_ok(g_s, g_t, k) -> bool:
    """The one-launch post-processing serves: 2..4 stages, student and teacher
    with equal Gram sizes k+3 <= W <= 63, k <= 8, on the GPU."""
    return (2 <= len(g_s) <= 4 and 1 <= k <= 8 and g_s[0].is_cuda and _ext.available()
            and all(fs.shape[-1] == ft.shape[-1] and k + 3 <= fs.shape[-1] <= 63
                    for fs, ft in zip(g_s, g_t)))


def kdsvd_native_ok(g_s, g_t) -> bool:
    """Every stage's SVD runs on the Gram eigensolver (graph-capturable)."""
    return all(_svd_native_ok(f) for f in list(g_s) + list(g_t))


def kdsvd_loss(g_s, g_t, k, native: bool | None = None, fused: bool | str | None = None):
    """`distillers/KDSVD.py:8-35`.  ``native`` (default: whenever the shapes
    allow): the SVDs through the Gram eigendecomposition (:class:`_GramEig`);
    else torch.linalg.svd (rocSOLVER, host-synchronising).  Singular vectors
    are defined up to sign; the native path's convention (largest component
    positive) differs from LAPACK's arbitrary one, so the teacher-side signs
    -- and with them the inter-stage RBF terms -- can differ from the
    reference (parity is pinned on sign-invariant quantities).

    ``fused`` (GPU): None/True -- :class:`_KdsvdNative` (everything native);
    "post" -- _GramEig + the fused post-processing; False -- PyTorch ops
    around the eigensolver."""
    if native is None:
        native = kdsvd_native_ok(g_s, g_t)
    if native and fused in (None, True) and kdsvd_native_full_ok(g_s, g_t, k):
        return _KdsvdNative.apply(int(k), len(g_s), *g_s, *g_t)
    if native and fused is not False and kdsvd_fused_ok(g_s, g_t, k):
        # fused="post": eigendecompositions through _GramEig, post-processing fused
        lts, vts, vss = [], [], []
        for f_s, f_t in zip(g_s, g_t):
            N, C, H, W = f_t.shape
            xt = f_t.detach().float().contiguous().reshape(N, C * H, W)
            N, C, H, W = f_s.shape
            xs = f_s.float().contiguous().reshape(N, C * H, W)
            _, vec_s, lam_t, vec_t = _GramEig.apply(xs, xt)
            lts.append(lam_t)
            vts.append(vec_t)
            vss.append(vec_s)
        return _KdsvdPost.apply(int(k), lts, vts, *vss)
    v_sb = v_tb = None
    losses = []
    for i, (f_s, f_t) in enumerate(zip(g_s, g_t)):
        if native and f_s.shape[-1] == f_t.shape[-1]:
            # student and teacher Grams diagonalised in one launch
            N, C, H, W = f_t.shape
            xt = f_t.detach().float().contiguous().reshape(N, C * H, W)
            N, C, H, W = f_s.shape
            xs = f_s.float().contiguous().reshape(N, C * H, W)
            lam_s, vec_s, lam_t, vec_t = _GramEig.apply(xs, xt)
            _, s_t, v_t = _svd_post(lam_t, vec_t, k, exact=True)
            _, _, v_s = _svd_post(lam_s, vec_s, k + 3, exact=True)
        else:
            svd = _svd_gram if native else _svd
            _, s_t, v_t = svd(f_t.detach(), k)
            _, _, v_s = svd(f_s, k + 3)
        v_s, v_t = _align_rsv(v_s, v_t)
        s_t = s_t.unsqueeze(1)
        v_t = v_t * s_t
        v_s = v_s * s_t
        if i > 0:
            s_rbf = torch.exp(-(v_s.unsqueeze(2) - v_sb.unsqueeze(1)).pow(2) / 8)
            t_rbf = torch.exp(-(v_t.unsqueeze(2) - v_tb.unsqueeze(1)).pow(2) / 8)
            l2 = (s_rbf - t_rbf.detach()).pow(2)
            l2 = torch.where(torch.isfinite(l2), l2, torch.zeros_like(l2))
            losses.append(l2.sum())
        v_tb, v_sb = v_t, v_s
    bsz = g_s[0].shape[0]
    return sum(l / bsz for l in losses)


# ---------------------------------------------------------------- VID
class _VIDNLL(torch.autograd.Function):
    """VID Gaussian NLL on the native kernels (csrc/feat.hip mda_vid_loss /
    mda_vid_bwd): one channel-sum pass + a one-block finalize forward, one
    elementwise pass backward (+ the per-channel log-scale gradient)."""

    @staticmethod
    def forward(ctx, pred, f_t, log_scale, eps):
        N, C, H, W = pred.shape
        M = N * H * W
        # S_c, then one partial row per block of the sums kernel (fixed-order sum)
        acc = torch.empty((1 + 512) * C, dtype=torch.float64, device=pred.device)
        loss = torch.empty(1, dtype=torch.float32, device=pred.device)
        ls = log_scale.detach().float().contiguous()
        _ext.call("mda_vid_loss", pred, f_t, ls, M, C, float(eps), acc, loss)
        ctx.save_for_backward(pred, f_t, ls, acc)
        ctx.meta = (M, C, float(eps), log_scale.dtype)
        return loss[0]

    @staticmethod
    def backward(ctx, go):
        pred, f_t, ls, acc = ctx.saved_tensors
        M, C, eps, lsdt = ctx.meta
        g = go.detach().float().reshape(1).contiguous()
        dpred = torch.empty_like(pred)
        dls = torch.empty(C, dtype=torch.float32, device=pred.device) if ctx.needs_input_grad[2] else None
        _ext.call("mda_vid_bwd", pred, f_t, ls, acc, g, M, C, eps, dpred, dls)
        return dpred, None, (dls.to(lsdt) if dls is not None else None), None


def _vid_native_ok(regressor, f_s, f_t) -> bool:
    if not (hip_enabled_for(f_s) and f_s.dim() == 4 and f_t.dim() == 4 and f_s.shape[2:] == f_t.shape[2:]):
        return False
    convs = [m for m in regressor if isinstance(m, nn.Conv2d)]
    return (len(convs) == 3 and all(c.bias is None and c.kernel_size == (1, 1) and c.groups == 1
                                    for c in convs)
            and all(c.out_channels % 8 == 0 and c.in_channels % 8 == 0 for c in convs)
            and f_t.shape[1] <= 2048)


def vid_loss(regressor, log_scale, f_s, f_t, eps=1e-5):
    """`distillers/VID.py:16-30`: Gaussian NLL with softplus variance.

    On the GPU the 1x1 -> ReLU -> 1x1 -> ReLU -> 1x1 regressor runs as three
    native conv launches (ReLU in the epilogue) and the NLL on
    :class:`_VIDNLL`; elsewhere the PyTorch formulation."""
    f_s, f_t = _pool_to_match(f_s, f_t)
    if _vid_native_ok(regressor, f_s, f_t):
        from .nn import conv_bn_act
        c1, c2, c3 = [m for m in regressor if isinstance(m, nn.Conv2d)]
        x = f_s.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        h, _ = conv_bn_act(x, c1, None, "relu")
        h, _ = conv_bn_act(h, c2, None, "relu")
        pred, _ = conv_bn_act(h, c3, None, "none")
        pred = pred.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ft = f_t.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        return _VIDNLL.apply(pred, ft, log_scale, eps)
    pred_mean = regressor(f_s).float()
    pred_var = F.softplus(log_scale.float()) + eps
    pred_var = pred_var.view(1, -1, 1, 1)
    nlp = 0.5 * ((pred_mean - f_t.float()) ** 2 / pred_var + torch.log(pred_var))
    return nlp.mean()


# ---------------------------------------------------------------- ReviewKD HCL (K9)
def hcl_loss(fstudent, fteacher):
    """`distillers/ReviewKD.py:11-28`: MSE at full resolution plus a 4/2/1
    average-pooled pyramid, weights 1, 1/2, 1/4, ..., normalised."""
    loss_all = 0.0
    for fs, ft in zip(fstudent, fteacher):
        fs = fs.float()
        ft = ft.float()
        h = fs.shape[2]
        loss = F.mse_loss(fs, ft, reduction="mean")
        cnt, tot = 1.0, 1.0
        for l in (4, 2, 1):
            if l >= h:
                continue
            tmpfs = F.adaptive_avg_pool2d(fs, (l, l))
            tmpft = F.adaptive_avg_pool2d(ft, (l, l))
            cnt /= 2.0
            loss = loss + F.mse_loss(tmpfs, tmpft, reduction="mean") * cnt
            tot += cnt
        loss = loss / tot
        loss_all = loss_all + loss
    return loss_all


# --------------------------------------------------------------------------
# fused HIP path of HCL (csrc/reviewkd.hip::mda_hcl_loss)

def _hcl_cpb(C, HW):
    # channels per block: ~8 K staged floats (~30 KB of LDS -> several blocks
    # per CU); power of two <= 32 (csrc/reviewkd.hip HCL_MAX_CPB)
    for cpb in (32, 16, 8, 4, 2, 1):
        if C % cpb == 0 and HW * cpb <= 8192:
            return cpb
    return 0


def hcl_native_ok(fstudent, fteacher) -> bool:
    from .backend import hip_enabled_for
    if not fstudent or len(fstudent) != len(fteacher) or len(fstudent) > 8:
        return False
    for a, b in zip(fstudent, fteacher):
        if not (hip_enabled_for(a) and a.dim() == 4 and a.shape == b.shape
                and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16):
            return False
        if _hcl_cpb(a.shape[1], a.shape[2] * a.shape[3]) == 0:
            return False
    return True


class _HCL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, warmup, epoch, n, *tensors):
        import numpy as np
        from . import _ext
        fs, ft = tensors[:n], tensors[n:]
        rows, grads, nblk, lds = [], [], 0, 0
        keep = []
        for a, b in zip(fs, ft):
            a = a.contiguous(memory_format=torch.channels_last)
            b = b.contiguous(memory_format=torch.channels_last)
            keep += [a, b]
            N, C, H, W = a.shape
            cpb = _hcl_cpb(C, H * W)
            g = torch.empty_like(a, memory_format=torch.channels_last)
            grads.append(g)
            nb = N * (C // cpb)
            rows.append([a.data_ptr(), b.data_ptr(), g.data_ptr(), N, H, W, C, cpb, nblk, nb])
            nblk += nb
            lds = max(lds, (H * W + H * 7) * cpb)  # staged d + row-bin sums
        table = np.asarray(rows, dtype=np.int64)
        dev = fs[0].device
        partial = torch.empty(nblk, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        ep = epoch if (epoch is not None and warmup and warmup > 0) else None
        _ext.call("mda_hcl_loss", table.ctypes.data, len(rows), nblk, lds, partial, float(weight),
                  ep, float(warmup or 0.0), loss)
        ctx.save_for_backward(*grads)
        ctx.n = n
        return loss.reshape(())

    @staticmethod
    def backward(ctx, go):
        from . import _ext
        grads = ctx.saved_tensors
        a = go.float().reshape(1).contiguous()
        outs = []
        for g in grads:
            o = torch.empty_like(g)
            _ext.call("mda_axpby", 1, a, g, None, None, o, g.numel())
            outs.append(o)
        return (None, None, None, None, *outs, *([None] * ctx.n))


def hcl_loss_weighted(fstudent, fteacher, weight, epoch=None, warmup=0.0):
    """``weight * min(epoch / warmup, 1) * hcl_loss(fstudent, fteacher)`` (teacher detached).

    On the GPU with bf16 features this is ONE fused launch (+ a tiny
    finalize) for all levels, forward value and gradient together.
    """
    ft = [t.detach() for t in fteacher]
    if hcl_native_ok(fstudent, ft) and (epoch is None or isinstance(epoch, torch.Tensor)):
        ep = epoch
        if ep is not None and (ep.dtype != torch.float32 or ep.device != fstudent[0].device):
            ep = ep.to(device=fstudent[0].device, dtype=torch.float32)
        return _HCL.apply(float(weight), float(warmup or 0.0), ep, len(fstudent), *fstudent, *ft)
    f = float(weight)
    if epoch is not None and warmup and warmup > 0:
        f = f * (torch.clamp(epoch.float() / float(warmup), max=1.0)
                 if isinstance(epoch, torch.Tensor) else min(float(epoch) / float(warmup), 1.0))
    return f * hcl_loss(fstudent, ft)
