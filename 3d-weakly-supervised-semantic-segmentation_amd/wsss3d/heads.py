"""Task heads and losses around the encoder (`models/MultiLabelContrastive.py:7-101`,
`utils/loss.py:5-33`).

The training call is `model((x, text), istrain=True)` (train.py:69) and the
eval call `model(x)` -> per-point logits (N, 20) (train.py:106), computed with
the Linear on the level-0 voxel rows (no (N, C) per-point features; the
device accumulation of train.py:107 is wsss3d.evaluate).  The text
model of MultiLabelContrastive is looked up in the registry: TextTransformer
(wsss3d/text.py) is registered; CLIPTransformer needs pretrained CLIP weights
that are not available offline.  Scene features in training come from the
encoder's fused tail (per-scene means without the (N, C) tensor).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from .encoders import segment_mean
from .registry import LOSS_REGISTRY, MODEL_REGISTRY
from .synthetic import NUM_CLASSES


def point_logits(encoder, x, linear):
    """linear(encoder(x)) as per-point logits (N, 20): through the encoder's fused voxel-level head
    (SparseConvBase_.point_logits, no (N, C) feature tensor) when it has one."""
    fn = getattr(encoder, "point_logits", None)
    return fn(x, linear) if fn is not None else linear(encoder(x))


def _encoder(pc_config):
    cls, meta = MODEL_REGISTRY.get(pc_config.name)
    width = meta.get("embed_length", lambda m: m)(pc_config.m)
    return cls(**pc_config), width


@MODEL_REGISTRY.register()
class MultiLabel(nn.Module):
    """Scene-level multilabel classification (models/MultiLabelContrastive.py:50-70)."""

    def __init__(self, pc_config):
        super().__init__()
        self.pc_encoder, width = _encoder(pc_config)
        self.linear = nn.Linear(width, NUM_CLASSES)

    def forward(self, x, istrain=False):
        if not istrain:
            return point_logits(self.pc_encoder, x, self.linear)
        return self.linear(self.pc_encoder(x[0], True)), None


@MODEL_REGISTRY.register()
class FullySupervised(nn.Module):
    """Per-point logits + per-scene mean logits (models/MultiLabelContrastive.py:72-101)."""

    def __init__(self, pc_config):
        super().__init__()
        self.pc_encoder, width = _encoder(pc_config)
        self.linear = nn.Linear(width, NUM_CLASSES)

    def forward(self, x, istrain=False):
        if istrain:
            pc_input = x[0]
            logits = point_logits(self.pc_encoder, pc_input, self.linear)
            return segment_mean(logits, pc_input.batch_offsets), logits
        return point_logits(self.pc_encoder, x, self.linear)


@MODEL_REGISTRY.register()
class MultiLabelContrastive(nn.Module):
    """Point + text heads (models/MultiLabelContrastive.py:7-47).  The scene
    features are the encoder's training output (per-scene means, the
    reference's loop at :34-39, through the fused tail)."""

    def __init__(self, pc_config, text_config):
        super().__init__()
        self.pc_encoder, width = _encoder(pc_config)
        text_cls, _ = MODEL_REGISTRY.get(text_config.name)
        self.text_encoder = text_cls(**text_config)
        self.text_linear = nn.Linear(text_config.width, width)
        self.linear = nn.Linear(width, NUM_CLASSES)

    def forward(self, x, istrain=False):
        if not istrain:
            return point_logits(self.pc_encoder, x, self.linear)
        pc_input, (text, has_text) = x
        if has_text.size(0) > 0:
            bt, nt, length = text.size()
            tf = self.text_encoder(text.view(-1, length), as_dict=True)["x"].view(bt, nt, -1)
            text_feats = self.text_linear(tf)
        else:
            text_feats = -1
        global_feats = self.pc_encoder(pc_input, istrain=True)
        return self.linear(global_feats), (global_feats, text_feats, has_text)


@LOSS_REGISTRY.register()
def TextContrastive(pc: torch.Tensor, text: torch.Tensor, has_text):
    """utils/loss.py:5-18"""
    if has_text.size(0) == 0:
        return 0
    sim = text @ pc.T  # B', num_text, B
    labels = has_text[:, None].expand(-1, sim.size(1))
    return F.cross_entropy(sim.transpose(1, 2), labels)


@LOSS_REGISTRY.register()
def Classification(logits: torch.Tensor, labels: torch.Tensor):
    """utils/loss.py:20-33: scene level (B, C) multilabel soft margin, point
    level (N,) cross entropy ignoring -100."""
    if labels.ndim == 2:
        return F.multilabel_soft_margin_loss(logits, labels)
    keep = labels != -100
    return F.cross_entropy(logits[keep], labels[keep])
