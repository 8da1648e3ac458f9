"""Model zoo: stem-inclusive feature contract, staged forward, parameter counts."""
import pytest
import torch

from mdistiller_ddp_amd.models import (cifar_model_dict, tiny_imagenet_model_dict,
                                       imagenet_model_dict, check_staged_forward)

# parameter counts measured on the reference models
PARAMS_M = {"resnet32x4": 7.43, "resnet8x4": 1.23, "resnet56": 0.86, "resnet20": 0.28,
            "resnet110": 1.74, "wrn_40_2": 2.26, "wrn_16_2": 0.70, "vgg13": 9.46, "vgg8": 3.97,
            "MobileNetV2": 0.81, "ShuffleV1": 0.95, "ShuffleV2": 1.36, "ResNet50": 23.71,
            "ResNet18": 11.22}


@pytest.mark.parametrize("name", sorted(cifar_model_dict))
def test_cifar_model_contract(name):
    torch.manual_seed(0)
    m = cifar_model_dict[name][0](num_classes=100).eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        logits, f = m(x)
    assert logits.shape == (2, 100)
    feats, pre = f["feats"], f["preact_feats"]
    assert len(feats) == len(pre) and len(feats) >= 4
    chans = m.get_stage_channels()
    assert len(chans) == len(feats), (name, chans, [t.shape for t in feats])
    for t, c in zip(feats, chans):
        assert t.shape[0] == 2 and t.shape[1] == c
    assert f["pooled_feat"].shape[0] == 2
    if name in PARAMS_M:
        # the reference-shaped state_dict (channel-padded models, e.g. the
        # ShuffleNets, hold zero pad rows the reference has not)
        params = dict(m.named_parameters())
        n = sum(v.numel() for k, v in m.state_dict().items() if k in params) / 1e6
        assert abs(n - PARAMS_M[name]) < 0.01, (name, n)


@pytest.mark.parametrize("name", sorted(cifar_model_dict))
def test_staged_forward_equivalence(name):
    torch.manual_seed(0)
    m = cifar_model_dict[name][0](num_classes=100)
    res = check_staged_forward(m, torch.randn(2, 3, 32, 32))
    assert res["all"], res


def test_bn_before_relu_matches_stages():
    m = cifar_model_dict["resnet32x4"][0](num_classes=100)
    bns = m.get_bn_before_relu()
    assert [b.num_features for b in bns] == m.get_stage_channels()[1:]


@pytest.mark.parametrize("name", sorted(tiny_imagenet_model_dict))
def test_tiny_imagenet_models(name):
    m = tiny_imagenet_model_dict[name][0](num_classes=200).eval()
    with torch.no_grad():
        logits, f = m(torch.randn(2, 3, 64, 64))
    assert logits.shape == (2, 200)  # ShuffleV2 at 64^2 works (reference D8 crashes)


@pytest.mark.parametrize("name", ["ResNet18", "ResNet34", "ResNet50", "MobileNetV1"])
def test_imagenet_cnns(name):
    m = imagenet_model_dict[name](pretrained=False, num_classes=1000).eval()
    with torch.no_grad():
        logits, f = m(torch.randn(1, 3, 224, 224))
    assert logits.shape == (1, 1000)
    assert len(f["feats"]) == 5  # stem + 4 stages
    assert [t.shape[1] for t in f["feats"]] == m.get_stage_channels()
    res = check_staged_forward(m, torch.randn(1, 3, 96, 96))
    assert res["all"], res


def test_vit_tiny_forward():
    m = imagenet_model_dict["vit_tiny"](pretrained=False, num_classes=1000).eval()
    with torch.no_grad():
        logits, f = m(torch.randn(1, 3, 224, 224))
    assert logits.shape == (1, 1000)
    assert m.get_arch() == "transformer"


def test_vgg_and_mv2_fused_forms_match_the_reference_composition():
    """Round 6 moved VGG's / Tiny-ImageNet MobileNetV2's ReLU(6)s into the
    producing conv launch (returning the pre-activation too) and their heads
    onto ``pool_linear``: on the CPU the logits, features, pre-activations and
    pooled features equal the reference's F.relu / AdaptiveAvgPool2d / Linear
    composition exactly (reference models/cifar/vgg.py, mv2_tinyimagenet.py)."""
    import copy
    import torch.nn.functional as F
    from mdistiller_ddp_amd.models._seq import run_seq
    from mdistiller_ddp_amd.models.cifar import vgg
    from mdistiller_ddp_amd.models.cifar.mv2_tinyimagenet import mobilenetv2_tinyimagenet
    torch.manual_seed(0)
    m = vgg.vgg8_bn(num_classes=100).train()
    ref = copy.deepcopy(m)
    x = torch.randn(2, 3, 32, 32)
    logits, d = m(x)
    h, p0 = run_seq(ref.block0, x, want_preact=True)
    h = F.relu(h)
    feats, pres = [h], [p0]
    for i, (pool, block) in enumerate(((ref.pool0, ref.block1), (ref.pool1, ref.block2),
                                        (ref.pool2, ref.block3), (ref.pool3, ref.block4))):
        if i < 3 or h.shape[-1] > 4:
            h = pool(h)
        h, _ = run_seq(block, h)
        pres.append(h)
        h = F.relu(h)
        feats.append(h)
    avg = ref.pool4(h).reshape(2, -1)
    assert torch.equal(logits, ref.classifier(avg)) and torch.equal(d["pooled_feat"], avg)
    assert all(torch.equal(a, b) for a, b in zip(d["feats"], feats))
    assert all(torch.equal(a, b) for a, b in zip(d["preact_feats"], pres))

    m = mobilenetv2_tinyimagenet(num_classes=200).train()
    ref = copy.deepcopy(m)
    x = torch.randn(2, 3, 64, 64)
    logits, d = m(x)
    f0 = run_seq(ref.pre, x)[0]
    h = ref.stage1(F.relu6(f0))
    f1 = ref.stage2(h)
    f2 = ref.stage3(F.relu6(f1))
    f3 = ref.stage4(F.relu6(f2))
    h = ref.stage7(ref.stage6(ref.stage5(F.relu6(f3))))
    f4 = run_seq(ref.conv1, h)[0]
    avg = F.adaptive_avg_pool2d(f4, 1)
    assert torch.equal(logits, ref.conv2(avg).flatten(1))
    assert torch.equal(d["pooled_feat"], avg.flatten(1))
    assert all(torch.equal(a, F.relu6(b)) for a, b in zip(d["feats"], (f0, f1, f2, f3, f4)))
    assert all(torch.equal(a, b) for a, b in zip(d["preact_feats"], (f0, f1, f2, f3, f4)))
