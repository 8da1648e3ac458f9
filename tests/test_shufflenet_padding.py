"""ShuffleNetV1 with physically padded groups (models/cifar/shufflenet.py
BottleneckV1) is the reference network: loaded with the reference model's
state_dict it gives the reference's logits, features and parameter gradients
(stored once from `mdistiller/models/cifar/ShuffleNetv1.py` by
``scripts/gen_ref_fixtures.py``, fp64, a narrow groups-3 net with padded
18/20/30-channel groups) on the CPU path; the pad channels stay exactly zero
through SGD steps."""
import pytest
import torch

from mdistiller_ddp_amd.models.cifar.shufflenet import BottleneckV1, ShuffleNet, ShuffleV1
from tests import _fixtures as FX

CFG = {"out_planes": [120, 240, 480], "num_blocks": [2, 2, 2], "groups": 3}  # gen_ref_fixtures.SHUV1_CFG


def _ref_state():
    d = FX.load("ref_shufflenetv1")
    return {k[3:]: v.clone() for k, v in d.items() if k.startswith("sd/")}


def _ours():
    ours = ShuffleNet(CFG, num_classes=100)
    missing = ours.load_state_dict(_ref_state(), strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    return ours


def test_full_size_state_dict_is_the_reference_layout():
    """The full ShuffleV1 (240/480/960) has the reference checkpoint's keys and shapes."""
    import json
    import os
    with open(os.path.join(FX.DIR, "ref_shufflev1_shapes.json")) as f:
        ref = json.load(f)
    ours = {k: list(v.shape) for k, v in ShuffleV1(num_classes=100).state_dict().items()}
    assert ours == ref


def test_state_dict_shapes_are_the_reference():
    ref = _ref_state()
    ours = _ours().state_dict()
    assert ref.keys() == ours.keys()
    for k in ref:
        assert ref[k].shape == ours[k].shape, k
        torch.testing.assert_close(ours[k], ref[k], atol=0, rtol=0)


@pytest.mark.parametrize("train", [False, True])
def test_forward_backward_match_reference(train):
    # float64: the padded network is the same function to round-off (fp32 BN
    # at small maps x batch 2 amplifies summation-order noise)
    d = FX.load("ref_shufflenetv1")
    t = f"t{int(train)}"
    ours = _ours().double().train(train)
    lo, fo = ours(d["x"].clone())
    torch.testing.assert_close(lo, d[f"{t}/logits"], atol=1e-10, rtol=1e-10)
    # ours also returns the stem output as f0 (like the other CIFAR models)
    nref = sum(1 for k in d if k.startswith(f"{t}/feat"))
    assert len(fo["feats"]) == nref + 1
    for i in range(nref):
        torch.testing.assert_close(fo["feats"][i + 1], d[f"{t}/feat{i}"], atol=1e-10, rtol=1e-10)
    if not train:
        return
    lo.backward(d["t1/dlogits"].clone())
    # compare gradients in the reference's (unpadded) layout
    specs = ours._pad_entries()
    for n, p in ours.named_parameters():
        gr = p.grad
        if n in specs:
            dim, idx = specs[n]
            gr = gr.index_select(dim, torch.tensor(idx))
        torch.testing.assert_close(gr, d[f"grad/{n}"], atol=1e-10, rtol=1e-8, msg=n)


def test_pad_channels_stay_zero_under_sgd():
    ours = _ours()
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
