"""ShuffleNetV1 with physically padded groups (models/cifar/shufflenet.py
BottleneckV1) is the reference network: the reference's own model
(`mdistiller/models/cifar/ShuffleNetv1.py`, loaded read-only) and ours share a
state_dict and give the same logits, features and parameter gradients on the
CPU path; the pad channels stay exactly zero through SGD steps."""
import pytest
import torch

from mdistiller_ddp_amd.models.cifar.shufflenet import BottleneckV1, ShuffleV1
from tests import _refload as R

pytestmark = pytest.mark.skipif(not R.available(), reason="reference tree not mounted")


def _pair():
    ref_mod = R.load_model_module("cifar", "ShuffleNetv1")
    torch.manual_seed(0)

    # the reference's ShuffleNet leaves ModelBase.get_arch abstract, so its own
    # ShuffleV1() cannot be instantiated; supply it to build the same network
    class Ref(ref_mod.ShuffleNet):
        def get_arch(self):
            return "cnn"
    ref = Ref({"out_planes": [240, 480, 960], "num_blocks": [4, 8, 4], "groups": 3}, num_classes=100)
    ours = ShuffleV1(num_classes=100)
    missing = ours.load_state_dict(ref.state_dict(), strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    return ref, ours


def test_state_dict_shapes_are_the_reference():
    ref, ours = _pair()
    a, b = ref.state_dict(), ours.state_dict()
    assert a.keys() == b.keys()
    for k in a:
        assert a[k].shape == b[k].shape, k
        torch.testing.assert_close(a[k], b[k], atol=0, rtol=0)


@pytest.mark.parametrize("train", [False, True])
def test_forward_backward_match_reference(train):
    # float64: the padded network is the same function to round-off (fp32 BN
    # at 4x4 maps x batch 4 amplifies summation-order noise to ~1e-3)
    ref, ours = _pair()
    ref.double().train(train)
    ours.double().train(train)
    x = torch.randn(4, 3, 32, 32, dtype=torch.float64)
    lr, fr = ref(x)
    lo, fo = ours(x)
    torch.testing.assert_close(lo, lr, atol=1e-10, rtol=1e-10)
    # ours also returns the stem output as f0 (like the other CIFAR models)
    assert len(fo["feats"]) == len(fr["feats"]) + 1
    for a, b in zip(fr["feats"], fo["feats"][1:]):
        torch.testing.assert_close(b, a, atol=1e-10, rtol=1e-10)
    if not train:
        return
    g = torch.randn_like(lr)
    lr.backward(g)
    lo.backward(g)
    # compare gradients in the reference's (unpadded) layout
    rg = {n: p.grad for n, p in ref.named_parameters()}
    specs = ours._pad_entries()
    for n, p in ours.named_parameters():
        gr = p.grad
        if n in specs:
            dim, idx = specs[n]
            gr = gr.index_select(dim, torch.tensor(idx))
        torch.testing.assert_close(gr, rg[n], atol=1e-10, rtol=1e-8, msg=n)


def test_pad_channels_stay_zero_under_sgd():
    _, ours = _pair()
    ours.train()
    opt = torch.optim.SGD(ours.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    for _ in range(3):
        opt.zero_grad()
        lo, _ = ours(torch.randn(4, 3, 32, 32))
        lo.square().mean().backward()
        opt.step()
    for m in ours.modules():
        if isinstance(m, BottleneckV1):
            keep1 = torch.zeros(m.conv1.out_channels, dtype=torch.bool)
            keep1[m._idx1] = True
            keep3 = torch.zeros(m.conv2.out_channels, dtype=torch.bool)
            keep3[m._idx3] = True
            assert m.conv1.weight[~keep1].abs().max().item() == 0 if (~keep1).any() else True
            assert m.conv2.weight[~keep3].abs().max().item() == 0 if (~keep3).any() else True
            assert m.conv3.weight[:, m.real["m3"]:].abs().max().item() == 0 if m.real["m3"] < m.real["m3p"] else True
            for bn, keep in ((m.bn1, keep1), (m.bn2, keep3)):
                if (~keep).any():
                    assert bn.weight[~keep].abs().max().item() == 0
                    assert bn.bias[~keep].abs().max().item() == 0
