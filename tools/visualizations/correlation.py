#!/usr/bin/env python
"""Teacher-student logit discrepancy heatmap (reference
``tools/visualizations/correlation.ipynb``).

For each model the class-conditional mean logit matrix
``M[l] = mean of logits over validation samples with label l`` (C x C) is
computed; the heatmap shows ``|M_student - M_teacher|`` clipped at
``--max-diff`` (3.0 in the reference, a common scale across methods), and
the mean absolute difference is printed.

    python tools/visualizations/correlation.py -t resnet32x4 -s resnet8x4 \
        -c output/<exp>/student_best
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from common import base_parser, collect, load_model, save_figure, val_loader  # noqa: E402


def class_mean_logits(logits: np.ndarray, labels: np.ndarray, num_classes: int) -> np.ndarray:
    m = np.zeros((num_classes, logits.shape[1]), dtype=np.float64)
    np.add.at(m, labels, logits.astype(np.float64))
    cnt = np.bincount(labels, minlength=num_classes).astype(np.float64)[:, None]
    return m / np.maximum(cnt, 1.0)


def discrepancy(student_logits, teacher_logits, labels, num_classes):
    return np.abs(class_mean_logits(student_logits, labels, num_classes)
                  - class_mean_logits(teacher_logits, labels, num_classes))


def plot(diff: np.ndarray, max_diff: float, title: str = ""):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(7, 6))
    plt.imshow(np.clip(diff, 0, max_diff), vmin=0, vmax=max_diff, cmap="PuBuGn")
    plt.colorbar()
    plt.xticks([])
    plt.yticks([])
    if title:
        plt.title(title)
    return fig


def main(argv=None):
    p = base_parser(__doc__)
    p.add_argument("-t", "--teacher", required=True)
    p.add_argument("-s", "--student", required=True)
    p.add_argument("-c", "--ckpt", default="random", help="student checkpoint | random")
    p.add_argument("--teacher-ckpt", default="pretrain", help="checkpoint | pretrain | random")
    p.add_argument("--max-diff", type=float, default=3.0)
    args = p.parse_args(argv)
    import torch
    device = torch.device(args.device if (args.device != "cuda" or torch.cuda.is_available()) else "cpu")
    loader, ncls = val_loader(args.dataset, args.batch_size, args.synthetic, device)
    stu = load_model(args.dataset, args.student, args.ckpt, ncls)
    tea = load_model(args.dataset, args.teacher, args.teacher_ckpt, ncls)
    ls, _, labels = collect(stu, loader, device, args.max_batches)
    lt, _, labels_t = collect(tea, loader, device, args.max_batches)
    if not np.array_equal(labels, labels_t):
        raise RuntimeError("validation loader is not deterministic; cannot pair teacher/student")
    diff = discrepancy(ls, lt, labels, ncls)
    os.makedirs(args.out, exist_ok=True)
    tag = f"corr_{args.teacher}_{args.student}"
    np.save(os.path.join(args.out, tag + ".npy"), diff)
    save_figure(plot(diff, args.max_diff, f"{args.student} vs {args.teacher}: mean |diff| {diff.mean():.3f}"),
                os.path.join(args.out, tag + ".png"))
    print(f"mean |diff| = {diff.mean():.4f}  ->  {os.path.join(args.out, tag + '.png')}")
    return diff


if __name__ == "__main__":
    main()
