#!/usr/bin/env python
"""t-SNE of a student's pooled features on the validation split (reference
``tools/visualizations/tsne.ipynb``): one scatter, coloured by class.

    python tools/visualizations/tsne.py -m resnet8x4 -c output/<exp>/student_best
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402

from common import base_parser, collect, load_model, save_figure, val_loader  # noqa: E402


def tsne_embed(features: np.ndarray, seed: int = 0, perplexity: float = 30.0) -> np.ndarray:
    from sklearn.manifold import TSNE
    perplexity = min(perplexity, max(2.0, (features.shape[0] - 1) / 3.0))
    return TSNE(n_components=2, init="pca", random_state=seed,
                perplexity=perplexity).fit_transform(features)


def plot(emb: np.ndarray, labels: np.ndarray, num_classes: int, title: str = ""):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(6, 6))
    cmap = plt.get_cmap("tab20")
    for c in range(num_classes):
        sel = labels == c
        if sel.any():
            plt.scatter(emb[sel, 0], emb[sel, 1], color=cmap(c % 20), s=1, alpha=0.4)
    plt.xticks([])
    plt.yticks([])
    if title:
        plt.title(title)
    return fig


def main(argv=None):
    p = base_parser(__doc__)
    p.add_argument("-m", "--model", required=True)
    p.add_argument("-c", "--ckpt", default="random", help="checkpoint path | pretrain | random")
    p.add_argument("--seed", type=int, default=0)
    args = p.parse_args(argv)
    import torch
    device = torch.device(args.device if (args.device != "cuda" or torch.cuda.is_available()) else "cpu")
    loader, ncls = val_loader(args.dataset, args.batch_size, args.synthetic, device)
    model = load_model(args.dataset, args.model, args.ckpt, ncls)
    _, feats, labels = collect(model, loader, device, args.max_batches)
    emb = tsne_embed(feats, args.seed)
    os.makedirs(args.out, exist_ok=True)
    tag = f"tsne_{args.model}"
    np.savez(os.path.join(args.out, tag + ".npz"), embedding=emb, labels=labels)
    save_figure(plot(emb, labels, ncls, f"{args.model} ({os.path.basename(args.ckpt)})"),
                os.path.join(args.out, tag + ".png"))
    print(os.path.join(args.out, tag + ".png"))
    return emb, labels


if __name__ == "__main__":
    main()
