"""Point-cloud encoder plugin surface (`models/SparseConvNet.py:10-229`).

`SparseConvBase_` keeps the reference's contract: construct with the class's
own name plus the YAML `pointcloud_model` keys, `getEncoder(**kw)` returns a
callable over `[coords, feats]`, `forward(x, istrain)` returns per-point
features `(N, C)` (or per-scene means `(B, C)` when `istrain`).  Every encoder
registered by the reference is registered here with the same name and
`embed_length`, built on the `sparseconvnet` namespace of this package, so a
reference `models/SparseConvNet.py` also runs unchanged on top of it.
"""
from __future__ import annotations

from typing import List

import torch
from torch import nn

import sparseconvnet as scn
from sparseconvnet.ops import PointLogitsFunction, SceneMeanFunction

from .registry import MODEL_REGISTRY


def segment_mean(feats: torch.Tensor, batch_offsets) -> torch.Tensor:
    """Mean of feats over the point ranges [off[b], off[b+1]) -> (B, C)
    (`models/SparseConvNet.py:20-26`).  One reduction per scene, as the
    reference does: a single fp32 index_add over ~2e5 points per scene was
    measured 1e-4 off the fp64 mean (atomic accumulation into one row),
    while torch's tree reduction stays at ~1e-7."""
    off = [int(o) for o in batch_offsets]
    return torch.stack([feats[off[b]:off[b + 1]].mean(0) for b in range(len(off) - 1)])


class SparseConvBase_(nn.Module):
    """Subclasses redefine getEncoder; encode/postProcessing are optional."""

    def getEncoder(self, *args, **kwarg):
        return None

    def encode(self, input: List[torch.Tensor]):
        return self.encoder(input)

    def postProcessing(self, out_feats: torch.Tensor, batch_offsets: list):
        return segment_mean(out_feats, batch_offsets)

    def __init__(self, name: str, *args, **kwarg):
        super().__init__()
        if name != type(self).__name__:
            raise AssertionError(f"encoder name {name!r} does not match class {type(self).__name__!r}")
        self.encoder = self.getEncoder(*args, **kwarg)

    @staticmethod
    def _inputs(x):
        if not isinstance(x, dict):
            raise AssertionError(f"batch data type unsupported. Expected EasyDict, got {type(x)}. ")
        coords, feats = x["coords"], x["feature"]
        if coords.size(0) != feats.size(0):
            raise AssertionError(f"Coords and feats not aligned! coords's batchsize is {coords.size(0)} "
                                 f"while feats' is {feats.size(0)}. ")
        return coords, feats

    def forward(self, x, istrain=False):
        coords, feats = self._inputs(x)
        if istrain and self._fusable():
            return self._encode_scene_means(coords, feats, x["batch_offsets"])
        out = self.encode([coords, feats])
        return self.postProcessing(out, x["batch_offsets"]) if istrain else out

    def point_logits(self, x, linear: nn.Linear):
        """`linear(self(x))` -- the per-point logits of the reference's eval call (train.py:106;
        models/MultiLabelContrastive.py:43-45, 84-101) -- with the Linear applied to the level-0 voxel rows
        before the OutputLayer's gather (ops.PointLogitsFunction): the (N, C)
        per-point feature tensor (N x 896 floats for SparseConvFCNet m=32) is never formed.  Same values up to
        fp32 rounding (the gather is a copy); encoders that override encode/postProcessing take the per-point
        path."""
        coords, feats = self._inputs(x)
        if not self._fusable():
            return linear(self.encode([coords, feats]))
        t = self.encoder[:-1]([coords, feats])
        return PointLogitsFunction.apply(t.features, linear.weight, linear.bias, t.metadata.input)

    # ---------------------------------------------------------------- fused tail
    def _fusable(self):
        """The default encode/postProcessing over a Sequential ending in an
        OutputLayer (every registered encoder): the training output can skip
        the (N, C) per-point tensor."""
        enc = self.encoder
        return (type(self).encode is SparseConvBase_.encode
                and type(self).postProcessing is SparseConvBase_.postProcessing
                and isinstance(enc, scn.Sequential) and len(enc) > 1 and isinstance(enc[-1], scn.OutputLayer))

    def _encode_scene_means(self, coords, feats, batch_offsets):
        """Per-scene means straight from the level-0 voxel rows
        (ops.SceneMeanFunction).  Valid when scene b is exactly the points of
        batch id b: batch column non-decreasing and the first/last point of
        every range carrying its index; otherwise the per-point path runs.
        The check compares the offsets with the scene starts the InputLayer
        read back together with its voxel count (InputRules.scene_ranges_match),
        so this path issues no device-to-host read of its own."""
        B = len(batch_offsets) - 1
        t = self.encoder[:-1]([coords, feats])
        rules = t.metadata.input
        if not rules.scene_ranges_match(batch_offsets):
            return self.postProcessing(self.encoder[-1](t), batch_offsets)
        lvl = t.metadata.level(int(t.spatial_size[0]))
        out, _ = SceneMeanFunction.apply(t.features, lvl, rules, B)
        return out


def _wrap(dimension, full_scale, m, make_body, out_planes):
    """InputLayer(mode 4) -> SubM(3 -> m) -> body -> BNReLU -> OutputLayer:
    the frame every reference encoder uses.  Modules are created in the
    reference's order (the first SubM before the body), so a seeded init draws
    the same weights as the reference's getEncoder."""
    inp = scn.InputLayer(dimension, full_scale, mode=4)
    first = scn.SubmanifoldConvolution(dimension, 3, m, 3, False)
    return scn.Sequential(inp, first, make_body(), scn.BatchNormReLU(out_planes), scn.OutputLayer(dimension))


def _levels(m, depth=7):
    return [(i + 1) * m for i in range(depth)]


@MODEL_REGISTRY.register(embed_length=lambda m: m)
class SparseConvUNet(SparseConvBase_):
    """models/SparseConvNet.py:57-71"""

    def getEncoder(self, m, dimension, full_scale, block_reps, residual_blocks):
        return _wrap(dimension, full_scale, m, lambda: scn.UNet(dimension, block_reps, _levels(m), residual_blocks), m)


@MODEL_REGISTRY.register(embed_length=lambda m: 7 * (7 + 1) * m // 2)
class SparseConvFCNet(SparseConvBase_):
    """models/SparseConvNet.py:73-88; output = all 7 levels joined (28m)."""

    def getEncoder(self, m, dimension, full_scale, block_reps, residual_blocks, depth: int = 7,
                   downsample=[2, 2]):
        planes = _levels(m, depth)
        return _wrap(dimension, full_scale, m, lambda: scn.FullyConvolutionalNet(
            dimension, block_reps, planes, residual_blocks, downsample=downsample), sum(planes))


@MODEL_REGISTRY.register(embed_length=lambda m: sum([m, 64, 128, 192, 256]))
class SparseConvFCNetNarrow(SparseConvBase_):
    """models/SparseConvNet.py:90-105"""

    def getEncoder(self, m, dimension, full_scale, block_reps, residual_blocks,
                   nPlanes: List[int] = [64, 128, 192, 256], downsample=[2, 2]):
        planes = [m] + list(nPlanes)
        return _wrap(dimension, full_scale, m, lambda: scn.FullyConvolutionalNet(
            dimension, block_reps, planes, residual_blocks, downsample=downsample), sum(planes))


class _DirectUpPool(SparseConvBase_):
    """Shared body of the FCNEncoder variants (models/SparseConvNet.py:107-211):
    only the deepest level's features come back up through UnPooling."""

    default_planes: List[int] = [64, 128, 192, 256]
    default_downsample = [2, 2]

    def FCNEncoder(self, dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2]):
        return scn.FullyConvolutionalNetEncoder(dimension, reps, nPlanes, residual_blocks, downsample)

    def getEncoder(self, m, dimension, full_scale, block_reps, residual_blocks, nPlanes=None, downsample=None):
        planes = [m] + list(self.default_planes if nPlanes is None else nPlanes)
        ds = self.default_downsample if downsample is None else downsample
        return _wrap(dimension, full_scale, m, lambda: self.FCNEncoder(
            dimension, block_reps, planes, residual_blocks, downsample=ds), planes[-1])


@MODEL_REGISTRY.register(embed_length=lambda m: 256)
class SparseConvFCNetDirectUpPool(_DirectUpPool):
    pass


@MODEL_REGISTRY.register(embed_length=lambda m: 128)
class SparseConvFCNetDirectUpPoolLight(_DirectUpPool):
    default_planes = [32, 64, 96, 128]
    default_downsample = [4, 4]


@MODEL_REGISTRY.register(embed_length=lambda m: 256)
class SparseConvFCNetIndirectUpPool(_DirectUpPool):
    """Registered but unconstructible in the reference (it calls a
    non-existent self.FCNEncoder, models/SparseConvNet.py:214-229); here it
    gets the shared FCNEncoder so the name resolves to a working model."""


@MODEL_REGISTRY.register(embed_length=lambda m: 7 * m)
class SparseConvFCNetEncoder(SparseConvBase_):
    """Named in README.md:28 and config/3DUNetWithText_scannet_test.yaml:19 but
    never registered by the reference; built as Function_test.py:166-232's
    `FullyConvolutionalNetEncoder` over [m..7m] + BatchNormReLU(7m)."""

    def getEncoder(self, m, dimension, full_scale, block_reps, residual_blocks, depth: int = 7,
                   downsample=[2, 2]):
        planes = _levels(m, depth)
        return _wrap(dimension, full_scale, m, lambda: scn.FullyConvolutionalNetEncoder(
            dimension, block_reps, planes, residual_blocks, downsample), planes[-1])
