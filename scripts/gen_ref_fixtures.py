#!/usr/bin/env python
"""Generate the reference-parity fixtures once (``tests/fixtures/``).

Runs the reference's own loss functions, DOT optimizer and ShuffleNetV1
(read-only sources under ``$MDA_REFERENCE``, default /root/reference) on
fixed-seed inputs and stores inputs, outputs and gradients as safetensors.
The test suite only LOADS these files (``tests/test_parity_reference.py``,
``tests/test_shufflenet_padding.py``): no reference code runs inside a test
process.  Re-run after changing an input here:

    python scripts/gen_ref_fixtures.py
"""
import importlib.util
import os
import sys
import types

import torch
import torch.nn as nn
from safetensors.torch import save_file

REF = os.environ.get("MDA_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "fixtures")


def _pkg(name, path):
    if name not in sys.modules:
        pkg = types.ModuleType(name)
        pkg.__path__ = [path]
        sys.modules[name] = pkg


def _exec(full, path):
    spec = importlib.util.spec_from_file_location(full, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[full] = m
    spec.loader.exec_module(m)
    return m


def ref(kind, mod):
    base = os.path.join(REF, "mdistiller", kind)
    _pkg(f"_r_{kind}", base)
    return _exec(f"_r_{kind}.{mod}", os.path.join(base, mod + ".py"))


def ref_model(sub, mod):
    models = os.path.join(REF, "mdistiller", "models")
    _pkg("_r_models", models)
    if "_r_models._base" not in sys.modules:
        _exec("_r_models._base", os.path.join(models, "_base.py"))
    _pkg(f"_r_models.{sub}", os.path.join(models, sub))
    return _exec(f"_r_models.{sub}.{mod}", os.path.join(models, sub, mod + ".py"))


def grads_of(fn, tensors, nstudent):
    ts = [t.clone().requires_grad_(i < nstudent) for i, t in enumerate(tensors)]
    loss = fn(*ts)
    loss.sum().backward()
    return loss.detach().reshape(()), [t.grad for t in ts[:nstudent]]


def put_case(d, name, tensors, nstudent, fn):
    loss, gs = grads_of(fn, tensors, nstudent)
    for i, t in enumerate(tensors):
        d[f"{name}/in{i}"] = t.contiguous()
    d[f"{name}/loss"] = loss
    for i, g in enumerate(gs):
        d[f"{name}/grad{i}"] = g.contiguous()


def losses():
    d = {}
    KD, DKD = ref("distillers", "KD"), ref("distillers", "DKD")
    torch.manual_seed(0)
    put_case(d, "kd", [torch.randn(16, 100) * 3, torch.randn(16, 100) * 3], 1,
             lambda a, b: KD.kd_loss(a, b, 4.0))
    torch.manual_seed(1)
    s, t = torch.randn(16, 100) * 3, torch.randn(16, 100) * 3
    y = torch.randint(0, 100, (16,))
    d["dkd/target"] = y
    put_case(d, "dkd", [s, t], 1, lambda a, b: DKD.dkd_loss(a, b, y, 1.0, 8.0, 4.0))
    torch.manual_seed(2)
    B, C, T = 8, 37, 4.0
    s = (torch.randn(B, C) * 3).double()
    t = (torch.randn(B, C) * 3).double()
    y = torch.randint(0, C, (B,))
    d["dkd64/target"] = y
    put_case(d, "dkd64", [s, t], 1, lambda a, b: DKD.dkd_loss(a, b, y, 1.0, 8.0, T))

    AT = ref("distillers", "AT")
    torch.manual_seed(3)
    fs = [torch.randn(4, 8, 16, 16), torch.randn(4, 16, 8, 8)]
    ft = [torch.randn(4, 32, 16, 16), torch.randn(4, 64, 4, 4)]
    put_case(d, "at", fs + ft, 2, lambda a, b, c, e: AT.at_loss([a, b], [c, e], 2))

    NST = ref("distillers", "NST")
    torch.manual_seed(4)
    put_case(d, "nst", [torch.randn(4, 8, 8, 8), torch.randn(4, 16, 8, 8)], 1,
             lambda a, b: NST.nst_loss([a], [b]))
    torch.manual_seed(5)
    put_case(d, "nst_sq", [torch.randn(4, 16, 8, 8), torch.randn(4, 16, 8, 8)], 1,
             lambda a, b: NST.nst_loss([a], [b]))

    PKT, SP, RKD = ref("distillers", "PKT"), ref("distillers", "SP"), ref("distillers", "RKD")
    torch.manual_seed(5)
    put_case(d, "pkt", [torch.randn(16, 64), torch.randn(16, 32)], 1, PKT.pkt_loss)
    torch.manual_seed(6)
    put_case(d, "sp", [torch.randn(8, 16, 4, 4), torch.randn(8, 32, 4, 4)], 1,
             lambda a, b: SP.sp_loss([a], [b]))
    for sq in (False, True):
        torch.manual_seed(7)
        put_case(d, f"rkd_{int(sq)}", [torch.randn(10, 32), torch.randn(10, 64)], 1,
                 lambda a, b: RKD.rkd_loss(a, b, sq, 1e-12, 25, 50))

    KDSVD = ref("distillers", "KDSVD")
    torch.manual_seed(8)
    fs = [torch.randn(4, 8, 8, 8), torch.randn(4, 16, 4, 4)]
    ft = [torch.randn(4, 8, 8, 8), torch.randn(4, 16, 4, 4)]
    for i, f in enumerate(fs + ft):
        d[f"kdsvd/in{i}"] = f
    d["kdsvd/loss"] = KDSVD.kdsvd_loss(fs, ft, 1).reshape(())
    ref_svd = KDSVD.svd

    def svd_fixed(feat, n=1):  # deterministic singular-vector signs
        u, s_, v = ref_svd(feat, n)
        idx = v.abs().argmax(dim=1, keepdim=True)
        return u, s_, v * torch.where(v.gather(1, idx) < 0, -1.0, 1.0)
    KDSVD.svd = svd_fixed
    d["kdsvd/loss_signfix"] = KDSVD.kdsvd_loss(fs, ft, 1).reshape(())
    KDSVD.svd = ref_svd

    VID = ref("distillers", "VID")
    torch.manual_seed(9)
    reg = nn.Sequential(nn.Conv2d(8, 16, 1, bias=False), nn.ReLU(), nn.Conv2d(16, 16, 1, bias=False))
    ls = nn.Parameter(torch.randn(16))
    fs, ft = torch.randn(4, 8, 8, 8), torch.randn(4, 16, 4, 4)
    d["vid/w0"], d["vid/w2"] = reg[0].weight.detach().clone(), reg[2].weight.detach().clone()
    d["vid/log_scale"], d["vid/fs"], d["vid/ft"] = ls.detach().clone(), fs, ft
    d["vid/loss"] = VID.vid_loss(reg, ls, fs, ft, 1e-5).detach().reshape(())

    RV = ref("distillers", "ReviewKD")
    torch.manual_seed(10)
    fs = [torch.randn(2, 8, 8, 8), torch.randn(2, 16, 1, 1), torch.randn(2, 4, 16, 16)]
    ft = [torch.randn_like(f) for f in fs]
    for i, f in enumerate(fs + ft):
        d[f"hcl/in{i}"] = f
    d["hcl/loss"] = RV.hcl_loss(fs, ft).reshape(())

    OFD = ref("distillers", "OFD")
    torch.manual_seed(11)
    s, t = torch.randn(4, 8, 4, 4), torch.randn(4, 8, 4, 4)
    m = torch.randn(1, 8, 1, 1) - 1
    d["ofd/s"], d["ofd/t"], d["ofd/m"] = s, t, m
    d["ofd/loss"] = OFD.feat_loss(s, t, m).reshape(())

    CRD = ref("distillers", "CRD")
    torch.manual_seed(12)
    x = torch.rand(8, 33) * 1e-3
    d["crd/x"], d["crd/contrast_loss"] = x, CRD.ContrastLoss(500)(x).reshape(())
    N, D, K = 200, 16, 31
    torch.manual_seed(13)
    stdv = 1.0 / (D / 3) ** 0.5
    mem1 = torch.rand(N, D) * 2 * stdv - stdv
    mem2 = torch.rand(N, D) * 2 * stdv - stdv
    theirs = CRD.ContrastMemory.__new__(CRD.ContrastMemory)
    nn.Module.__init__(theirs)
    theirs.n_lem, theirs.K = N, K
    theirs.register_buffer("params", torch.tensor([K, 0.07, -1, -1, 0.5]))
    theirs.register_buffer("memory_v1", mem1.clone())
    theirs.register_buffer("memory_v2", mem2.clone())
    v1 = nn.functional.normalize(torch.randn(8, D), dim=1)
    v2 = nn.functional.normalize(torch.randn(8, D), dim=1)
    y = torch.arange(8) * 3
    idx = torch.randint(0, N, (8, K + 1))
    idx[:, 0] = y
    a1, a2 = theirs(v1, v2, y, idx)
    d.update({"crdmem/mem1": mem1, "crdmem/mem2": mem2, "crdmem/v1": v1, "crdmem/v2": v2,
              "crdmem/y": y, "crdmem/idx": idx, "crdmem/out1": a1.squeeze(-1).detach(),
              "crdmem/out2": a2.squeeze(-1).detach(), "crdmem/mem1_after": theirs.memory_v1.clone(),
              "crdmem/mem2_after": theirs.memory_v2.clone(), "crdmem/params": theirs.params.float().clone()})

    DOT = ref("engine", "dot")
    for reach in ("all", "mixed"):
        torch.manual_seed(14)
        shapes = [(5, 3), (7,), (4, 4), (3,)]
        p_ref = [nn.Parameter(torch.randn(s)) for s in shapes]
        for i, p in enumerate(p_ref):
            d[f"dot_{reach}/p{i}_init"] = p.detach().clone()
        mu, delta, lr, wd = 0.9, 0.075, 0.05, 5e-4
        opt = DOT.DistillationOrientedTrainer(p_ref, lr=lr, momentum=mu - delta,
                                              momentum_kd=mu + delta, weight_decay=wd)
        has_t = [True] * 4 if reach == "all" else [True, True, False, True]
        has_k = [True] * 4 if reach == "all" else [True, False, True, True]
        for step in range(5):
            gt = [torch.randn(s) for s in shapes]
            gk = [torch.randn(s) for s in shapes]
            for i in range(4):
                d[f"dot_{reach}/s{step}_gt{i}"] = gt[i]
                d[f"dot_{reach}/s{step}_gk{i}"] = gk[i]
            opt.zero_grad(set_to_none=True)
            for p, g, k in zip(p_ref, gk, has_k):
                p.grad = g.clone() if k else None
            opt.step_kd()
            opt.zero_grad(set_to_none=True)
            for p, g, t in zip(p_ref, gt, has_t):
                p.grad = g.clone() if t else None
            opt.step()
            for i, p in enumerate(p_ref):
                d[f"dot_{reach}/s{step}_p{i}"] = p.detach().clone()
    return d


# a narrow ShuffleNetV1 with the real network's structure: groups 3, 18/20/30-
# channel groups that the padded model rounds up, downsampling and residual
# blocks in every stage (the full 240/480/960 net is ~25 MB of fixtures)
SHUV1_CFG = {"out_planes": [120, 240, 480], "num_blocks": [2, 2, 2], "groups": 3}


def shufflenet():
    """Reference ShuffleNetV1 (groups 3, one block per stage: every block type
    and padding case, small enough to store) in float64: state_dict, a batch,
    logits / features in eval and train mode, and train-mode gradients."""
    mod = ref_model("cifar", "ShuffleNetv1")

    class Ref(mod.ShuffleNet):  # the snapshot leaves get_arch abstract
        def get_arch(self):
            return "cnn"
    torch.manual_seed(0)
    net = Ref(SHUV1_CFG, num_classes=100)
    # the fp32 init is exact in fp32: the state dict is stored fp32, the net runs fp64
    d = {f"sd/{k}": v.clone().contiguous() for k, v in net.state_dict().items()}
    net.double()
    torch.manual_seed(1)
    x = torch.randn(2, 3, 32, 32, dtype=torch.float64)
    d["x"] = x
    for train in (False, True):
        net.train(train)
        for p in net.parameters():
            p.grad = None
        logits, feats = net(x)
        d[f"t{int(train)}/logits"] = logits.detach().clone()
        for i, f in enumerate(feats["feats"]):
            d[f"t{int(train)}/feat{i}"] = f.detach().clone()
        if train:
            torch.manual_seed(2)
            g = torch.randn_like(logits)
            d["t1/dlogits"] = g
            logits.backward(g)
            for n, p in net.named_parameters():
                d[f"grad/{n}"] = p.grad.clone()
    return d


def shufflenet_full_shapes():
    """key -> shape of the full-size reference ShuffleV1 state dict (the
    checkpoint-loading contract of models/cifar/shufflenet.py)."""
    mod = ref_model("cifar", "ShuffleNetv1")

    class Ref(mod.ShuffleNet):
        def get_arch(self):
            return "cnn"
    net = Ref({"out_planes": [240, 480, 960], "num_blocks": [4, 8, 4], "groups": 3}, num_classes=100)
    return {k: list(v.shape) for k, v in net.state_dict().items()}


if __name__ == "__main__":
    import json
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "ref_shufflev1_shapes.json"), "w") as f:
        json.dump(shufflenet_full_shapes(), f, indent=0, sort_keys=True)
    a = losses()
    save_file(a, os.path.join(OUT, "ref_losses.safetensors"))
    b = shufflenet()
    save_file(b, os.path.join(OUT, "ref_shufflenetv1.safetensors"))
    for f in ("ref_losses.safetensors", "ref_shufflenetv1.safetensors"):
        print(f, os.path.getsize(os.path.join(OUT, f)))
