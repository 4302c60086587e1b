"""Vision Transformer (BASELINE.json config #5: ViT-Base/16 ASGD bf16).

Not in the reference (no sequence models there).  ViT-B/16 at
224x224 = 197 tokens, D=768, 12 heads, MLP 3072, 86,567,656 parameters with a
1000-class head.  LayerNorm and tanh-GELU are native kernels
(``csrc/transformer.hip``), multi-head attention is one fused MFMA kernel per
direction on the qkv rows (``csrc/attention.hip``); every projection / MLP GEMM
(forward, data and weight gradient) runs on the native MFMA GEMM
(``csrc/gemm.hip`` via ``ops.linear``), the MLP as one fused autograd op whose
fc1 epilogue applies GELU and whose fc2 data-gradient epilogue applies GELU'.
Patch embedding is a stride-16 conv computed as one GEMM over gathered patch
rows (``ops.linear.patch_embed``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import layers as L
from ..ops import functional as DF
from ..ops.functional import compute_weight
from ..ops.linear import mlp, mlp_ok, patch_embed, patch_embed_ok


class LayerNorm(nn.LayerNorm):
    def forward(self, x):
        return DF.layer_norm(x, self.weight, self.bias, self.eps, self._slots(x))

    def _slots(self, x):
        if not (x.is_cuda and self.weight is not None and self.weight.requires_grad):
            return None
        n = DF.LN_SLOTS * 2 * x.shape[-1]
        slots = self.__dict__.get("_dmp_slots")
        if slots is None or slots.device != x.device or slots.numel() != n:
            slots = torch.zeros(n, dtype=torch.float32, device=x.device)
            self.__dict__["_dmp_slots"] = slots
        return slots

    def stream_forward(self, x):
        """(x, LayerNorm(x)) with x's later gradient formed in the LN backward."""
        return DF.stream_layer_norm(x, self.weight, self.bias, self.eps, self._slots(x))

    def add_forward(self, x, r):
        """(h, LayerNorm(h)) with h = x + r, fused (pre-norm residual add)."""
        return DF.add_layer_norm(x, r, self.weight, self.bias, self.eps, self._slots(x))


class PatchEmbed(L.Conv2d):
    """Stride = kernel conv returning tokens ``[B, N, D]``; a GEMM on patch rows
    when the weight is arena-backed (parameter layout unchanged: a Conv2d)."""

    def forward(self, x):
        p = self.kernel_size[0]
        if patch_embed_ok(x, self.weight, self.bias, p):
            return patch_embed(x, self.weight, self.bias, p)
        return super().forward(x).flatten(2).transpose(1, 2)


class Attention(nn.Module):
    def __init__(self, dim: int, heads: int):
        super().__init__()
        self.heads = heads
        self.qkv = L.Linear(dim, 3 * dim)
        self.proj = L.Linear(dim, dim)

    def forward(self, x):
        # fused MFMA attention on the qkv rows as they come out of the projection
        # (csrc/attention.hip); SDPA / matmul + native softmax elsewhere
        return self.proj(DF.attention_qkv(self.qkv(x), self.heads))


class Block(nn.Module):
    def __init__(self, dim: int, heads: int, mlp_ratio: float = 4.0):
        super().__init__()
        self.norm1 = LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, heads)
        self.norm2 = LayerNorm(dim, eps=1e-6)
        hidden = int(dim * mlp_ratio)
        self.fc1 = L.Linear(dim, hidden)
        self.fc2 = L.Linear(hidden, dim)

    def mlp(self, y):
        if mlp_ok(y, self.fc1, self.fc2):
            return mlp(y, self.fc1, self.fc2)       # GELU fused into the GEMM epilogues
        return self.fc2(DF.gelu(self.fc1(y)))

    def forward(self, x):
        x = x + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))

    def forward_fused(self, h, pending=None):
        """Residual stream ``h`` plus the previous block's unadded MLP output
        ``pending``: every residual add is fused into the LayerNorm that reads
        its result (add + norm1, add + norm2).  Returns ``(h, mlp_out)`` with
        ``mlp_out`` still to be added by the caller (next block / final norm)."""
        if pending is None:
            h, y = self.norm1.stream_forward(h)
        else:
            h, y = self.norm1.add_forward(h, pending)
        h, y = self.norm2.add_forward(h, self.attn(y))
        return h, self.mlp(y)


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int = 224, patch: int = 16, dim: int = 768, depth: int = 12,
                 heads: int = 12, mlp_ratio: float = 4.0, num_classes: int = 1000,
                 in_chans: int = 3):
        super().__init__()
        assert image_size % patch == 0
        self.patch = patch
        self.num_patches = (image_size // patch) ** 2
        self.patch_embed = PatchEmbed(in_chans, dim, kernel_size=patch, stride=patch)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, self.num_patches + 1, dim))
        self.blocks = nn.ModuleList(Block(dim, heads, mlp_ratio) for _ in range(depth))
        self.norm = LayerNorm(dim, eps=1e-6)
        self.head = L.Linear(dim, num_classes)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.trunc_normal_(self.cls_token, std=0.02)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        w = self.patch_embed.weight
        nn.init.uniform_(w, -1 / math.sqrt(w[0].numel()), 1 / math.sqrt(w[0].numel()))

    def forward(self, x):
        h = self.patch_embed(x)                       # [B, N, D]
        h = DF.vit_embed(h, self.cls_token, self.pos_embed)   # cat(cls, h) + pos
        pending = None
        for blk in self.blocks:
            h, pending = blk.forward_fused(h, pending)
        if pending is None:
            y = self.norm(h)
        else:
            _, y = self.norm.add_forward(h, pending)
        # class token rows read in place by the head GEMM (no gather / zero-fill copies)
        return self.head(DF.token_row(y, 0))


def vit_b16(num_classes: int = 1000, image_size: int = 224) -> VisionTransformer:
    return VisionTransformer(image_size=image_size, patch=16, dim=768, depth=12, heads=12,
                             num_classes=num_classes)


def vit_tiny(num_classes: int = 10, image_size: int = 32, patch: int = 4) -> VisionTransformer:
    """Small ViT for CPU tests and CIFAR-shaped smoke runs."""
    return VisionTransformer(image_size=image_size, patch=patch, dim=64, depth=2, heads=4,
                             num_classes=num_classes)
