"""Text branch of MultiLabelContrastive (BASELINE
config 5): the causal text transformer of `models/Transformer.py:64-120`.

Dense and standard, so it runs on torch's ROCm kernels (hipBLASLt GEMMs and
the fused scaled-dot-product attention) rather than hand-written HIP.
Parameter names and shapes follow the reference module tree
(`transformer.resblocks.<i>.attn.in_proj_weight`, `...mlp.c_fc`, `ln_final`,
`token_embedding`, `positional_embedding`), so its checkpoints load; the
attention itself is computed with `F.scaled_dot_product_attention(is_causal)`
instead of `nn.MultiheadAttention` with an additive -inf mask (same math:
the reference mask is exactly the causal one, `build_attention_mask`).

Inputs are token ids (B, L) with the end-of-text token the largest id of each
row (`text.argmax(-1)` picks its position, `:117`), as produced by
`wsss3d.tokenizer.text_transform(max_seq_len, cropped_texts)` (the reference's
fixed-shape tokenizer, `dataset/dataset_utils/text_transform_builder.py:33-76`).
context_length must equal the padded sequence length (the reference's
3DUNetWithText configs pad to max_seq_len = 120).
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn.functional as F
from torch import nn

from .registry import MODEL_REGISTRY


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class CausalSelfAttention(nn.Module):
    """Holds nn.MultiheadAttention's parameters under its names (in_proj_weight,
    in_proj_bias, out_proj) and computes causal attention with SDPA."""

    def __init__(self, d_model: int, n_head: int):
        super().__init__()
        self.n_head = n_head
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d_model, d_model))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d_model))
        self.out_proj = nn.Linear(d_model, d_model)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.out_proj.bias)

    def forward(self, x):  # x: (B, L, D)
        B, L, D = x.shape
        h = self.n_head
        q, k, v = F.linear(x, self.in_proj_weight, self.in_proj_bias).split(D, dim=-1)
        q, k, v = (t.view(B, L, h, D // h).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.out_proj(y.transpose(1, 2).reshape(B, L, D))


class ResidualAttentionBlock(nn.Module):
    def __init__(self, d_model: int, n_head: int):
        super().__init__()
        self.attn = CausalSelfAttention(d_model, n_head)
        self.ln_1 = nn.LayerNorm(d_model)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d_model, 4 * d_model)), ("gelu", QuickGELU()),
                                              ("c_proj", nn.Linear(4 * d_model, d_model))]))
        self.ln_2 = nn.LayerNorm(d_model)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int, use_checkpoint: bool = False):
        super().__init__()
        self.width, self.layers, self.use_checkpoint = width, layers, use_checkpoint
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads) for _ in range(layers)])
        # initialisation scales of models/Transformer.py:44-52
        proj_std = width ** -0.5 * (2 * layers) ** -0.5
        for blk in self.resblocks:
            nn.init.normal_(blk.attn.in_proj_weight, std=width ** -0.5)
            nn.init.normal_(blk.attn.out_proj.weight, std=proj_std)
            nn.init.normal_(blk.mlp.c_fc.weight, std=(2 * width) ** -0.5)
            nn.init.normal_(blk.mlp.c_proj.weight, std=proj_std)

    def forward(self, x):
        for blk in self.resblocks:
            if self.use_checkpoint and x.requires_grad:
                x = torch.utils.checkpoint.checkpoint(blk, x, use_reentrant=False)
            else:
                x = blk(x)
        return x


@MODEL_REGISTRY.register()
class TextTransformer(nn.Module):
    """`models/Transformer.py:64-120`: token + positional embedding, causal
    pre-LN transformer (heads = width // 64), final LayerNorm, the feature at
    the end-of-text position."""

    def __init__(self, name: str, context_length: int, width: int, layers: int, vocab_size: int,
                 use_checkpoint: bool = False):
        super().__init__()
        if name != type(self).__name__:
            raise AssertionError(f"text model name {name!r} does not match {type(self).__name__!r}")
        self.context_length, self.width = context_length, width
        self.transformer = Transformer(width, layers, width // 64, use_checkpoint)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, width))
        self.ln_final = nn.LayerNorm(width)
        self.token_embedding = nn.Embedding(vocab_size, width)
        nn.init.normal_(self.token_embedding.weight, std=0.02)
        nn.init.normal_(self.positional_embedding, std=0.01)

    def forward(self, text, *, as_dict=False):
        if text.size(1) != self.context_length:
            raise ValueError(f"TextTransformer: sequences of length {text.size(1)} but context_length "
                             f"{self.context_length}")
        x = self.token_embedding(text) + self.positional_embedding
        x = self.ln_final(self.transformer(x))
        x = x[torch.arange(x.size(0), device=x.device), text.argmax(dim=-1)]
        return {"x": x} if as_dict else x
