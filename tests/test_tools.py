"""CLI tools on CPU: tools/eval.py on a saved student checkpoint and the
ImageNet linear probe on a tiny synthetic set."""
import os

import torch

from mdistiller_ddp_amd.models import cifar_model_dict, imagenet_model_dict
from mdistiller_ddp_amd.engine.utils import save_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_eval_cli(tmp_path, monkeypatch):
    import tools.eval as ev
    monkeypatch.setenv("MDA_BACKEND", "torch")
    m = cifar_model_dict["resnet8"][0](num_classes=100)
    ck = tmp_path / "student_best"
    save_checkpoint({"model": m.state_dict()}, str(ck))
    top1, top5, loss = ev.main(["-m", "resnet8", "-c", str(ck), "-d", "cifar100", "-bs", "50",
                                "--synthetic", "--dtype", "fp32"])
    assert 0 <= top1 <= 100 and top5 >= top1 and loss > 0


def test_lineval_imagenet_synthetic(tmp_path):
    from mdistiller_ddp_amd.config import get_cfg
    from tools.lineval import imagenet as li
    exp = tmp_path / "proj" / "exp"
    (exp / "code").mkdir(parents=True)
    cfg = get_cfg()
    cfg.DATASET.TYPE = "imagenet"
    cfg.DISTILLER.STUDENT = "vit_tiny"
    (exp / "code" / "_cfg.yaml").write_text(cfg.dump())
    m = imagenet_model_dict["vit_tiny"](pretrained=False)
    save_checkpoint({"model": m.state_dict()}, str(exp / "student_best"))
    best = li.main(["proj/exp", "-t", "best", "-bs", "2", "-tbs", "2", "-e", "1", "--synthetic",
                    "--output-root", str(tmp_path), "-nw", "0"])
    assert best >= 0
    assert list((exp / "lineval").rglob("best.pt"))


def test_nyud_patches_to_depth():
    from tools.lineval.nyud import patches_to_depth
    x = torch.randn(2, 1 + 196, 256)
    assert patches_to_depth(x).shape == (2, 224, 224)


def test_visualization_class_mean_logits():
    import numpy as np
    from tools.visualizations.correlation import class_mean_logits, discrepancy
    logits = np.array([[1.0, 2.0], [3.0, 4.0], [5.0, 7.0]])
    labels = np.array([0, 0, 1])
    m = class_mean_logits(logits, labels, 3)
    assert np.allclose(m, [[2.0, 3.0], [5.0, 7.0], [0.0, 0.0]])
    assert np.allclose(discrepancy(logits, logits + 1.0, labels, 3)[:2], 1.0)


def test_visualization_tools_synthetic(tmp_path):
    import numpy as np
    from tools.visualizations import correlation, tsne
    out = str(tmp_path / "viz")
    emb, labels = tsne.main(["-m", "resnet8", "--synthetic", "--max-batches", "2", "-bs", "32",
                             "--device", "cpu", "-o", out])
    assert emb.shape == (labels.shape[0], 2) and np.isfinite(emb).all()
    diff = correlation.main(["-t", "resnet20", "-s", "resnet8", "--teacher-ckpt", "random",
                             "--synthetic", "--max-batches", "2", "-bs", "32", "--device", "cpu",
                             "-o", out])
    assert diff.shape == (100, 100)
    assert os.path.exists(os.path.join(out, "tsne_resnet8.png"))
    assert os.path.exists(os.path.join(out, "corr_resnet20_resnet8.png"))
