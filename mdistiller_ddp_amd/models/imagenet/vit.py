"""Vision Transformer students (vit_tiny/small/base/large, patch16, 224^2).

The reference subclasses ``timm``'s VisionTransformer (`imagenet/vit.py:17-189`);
timm is not available here (and the reference file fails to import),
so this is a self-contained implementation with timm's parameter names
(``patch_embed.proj``, ``cls_token``, ``pos_embed``, ``blocks.N.{norm1,attn.qkv,
attn.proj,norm2,mlp.fc1,mlp.fc2}``, ``norm``, ``head``) so timm checkpoints
load with ``strict=True``.  Attention is the in-tree MFMA flash-attention
kernel on the HIP path (``ops/attention.py``, head_dim 64: tiny / small /
base / large) and PyTorch SDPA elsewhere; at 197 tokens there is nothing to
shard.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...ops.attention import attention
from .._base import ModelBase


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size, self.patch_size = img_size, patch_size
        self.num_patches = (img_size // patch_size) ** 2
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


class Attention(nn.Module):
    def __init__(self, dim, num_heads, qkv_bias=True):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        # fused MFMA flash attention on the HIP path (ops/attention.py), SDPA elsewhere
        return self.proj(attention(self.qkv(x), self.num_heads))


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=True):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads, qkv_bias)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class VisionTransformer(nn.Module, ModelBase):
    arch = "transformer"

    def __init__(self, img_size=224, patch_size=16, in_chans=3, num_classes=1000, embed_dim=768,
                 depth=12, num_heads=12, mlp_ratio=4.0, qkv_bias=True, global_pool="token"):
        super().__init__()
        self.embed_dim = self.num_features = embed_dim
        self.global_pool = global_pool
        self.patch_embed = PatchEmbed(img_size, patch_size, in_chans, embed_dim)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.randn(1, self.patch_embed.num_patches + 1, embed_dim) * 0.02)
        self.blocks = nn.Sequential(*[Block(embed_dim, num_heads, mlp_ratio, qkv_bias) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.fc_norm = nn.Identity()
        self.head = nn.Linear(embed_dim, num_classes) if num_classes > 0 else nn.Identity()
        nn.init.trunc_normal_(self.cls_token, std=1e-6)
        self.apply(self._init)
        self.stage_channels = [embed_dim] * (depth + 1)

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)

    def activate(self, x):
        return x

    def forward_stem(self, x):
        x = self.patch_embed(x)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1)
        return x + self.pos_embed

    def get_layers(self):
        return self.blocks

    def forward_pool(self, x):
        x = self.norm(x)
        x = x[:, 1:].mean(1) if self.global_pool == "avg" else x[:, 0]
        return self.fc_norm(x)

    def get_head(self):
        return self.head

    def get_bn_before_relu(self):
        raise NotImplementedError("ViT has no BN-before-ReLU stage ends")

    def forward(self, x):
        x = self.forward_stem(x)
        feats = [x]
        for blk in self.blocks:
            x = blk(x)
            feats.append(x)
        pooled = self.forward_pool(x)
        return self.head(pooled), {"feats": feats, "preact_feats": list(feats), "pooled_feat": pooled}


def _create(name, pretrained, **kw):
    m = VisionTransformer(**kw)
    if pretrained:
        root = os.environ.get("MDA_PRETRAINED_DIR", "")
        path = os.path.join(root, f"{name}.pth")
        if not root or not os.path.exists(path):
            raise FileNotFoundError(f"pretrained ViT weights {path!r} not found (no network download)")
        sd = torch.load(path, map_location="cpu", weights_only=True)
        m.load_state_dict(sd.get("model", sd))
    return m


def vit_tiny_patch16_224(pretrained=False, **kw):
    return _create("vit_tiny_patch16_224", pretrained, patch_size=16, embed_dim=192, depth=12, num_heads=3, **kw)


def vit_small_patch16_224(pretrained=False, **kw):
    return _create("vit_small_patch16_224", pretrained, patch_size=16, embed_dim=384, depth=12, num_heads=6, **kw)


def vit_base_patch16_224(pretrained=False, **kw):
    return _create("vit_base_patch16_224", pretrained, patch_size=16, embed_dim=768, depth=12, num_heads=12, **kw)


def vit_large_patch16_224(pretrained=False, **kw):
    return _create("vit_large_patch16_224", pretrained, patch_size=16, embed_dim=1024, depth=24, num_heads=16, **kw)
