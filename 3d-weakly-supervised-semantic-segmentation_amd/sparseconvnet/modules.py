"""`scn.*` layer classes with SparseConvNet's constructor signatures.

Constructor arguments, parameter names/shapes and initialisation follow the
SCN 0.2 API that the reference calls (SURVEY.md §8(b) Layer 1; call sites
models/SparseConvNet.py:60-229, Function_test.py:35-86):

  weight of (Submanifold)Convolution/Deconvolution: (filter_volume, groups,
      nIn/groups, nOut/groups) ~ N(0, sqrt(2 / (nIn * filter_volume)))
  NetworkInNetwork weight: (nIn, nOut) ~ N(0, sqrt(2 / nIn))
  BatchNormalization: weight=1, bias=0, running_mean=0, running_var=1,
      eps=1e-4, momentum=0.9 (SCN convention: running = m*running + (1-m)*batch)

Containers index their children '0', '1', ... like nn.Sequential so that
state_dict keys follow the module tree.
"""
from __future__ import annotations

import math
import sys

import torch
from torch import nn

from . import ops
from .metadata import Metadata, prefetch, take_prefetched
from .sparseConvNetTensor import SparseConvNetTensor


def _pkg():
    return sys.modules[__package__]


def _count(macs, out_features):
    pkg = _pkg()
    pkg.forward_pass_multiplyAdd_count += int(macs)
    pkg.forward_pass_hidden_states += int(out_features.nelement())


def _cube(v, dimension, what):
    vals = v.tolist() if torch.is_tensor(v) else (list(v) if isinstance(v, (list, tuple)) else [v] * dimension)
    vals = [int(a) for a in vals]
    if len(vals) != dimension or any(a != vals[0] for a in vals):
        raise NotImplementedError(f"{what}: only cubic sizes are supported, got {vals}")
    return vals[0]


def _check_dim(dimension):
    if dimension != 3:
        raise NotImplementedError(f"mi3dsparse implements dimension=3 (got {dimension})")


class InputLayer(nn.Module):
    """[coords (N,4) int, features (N,C)] -> SparseConvNetTensor.

    mode (Function_test.py:37-43): 0/2 first occurrence, 1 last occurrence,
    3 sum, 4 average of the points that share a voxel."""

    def __init__(self, dimension, spatial_size, mode=3):
        super().__init__()
        _check_dim(dimension)
        self.dimension = dimension
        self.spatial_size = torch.LongTensor([_cube(spatial_size, dimension, "InputLayer")] * dimension)
        self.mode = int(mode)
        if self.mode not in (0, 1, 2, 3, 4):
            raise ValueError(f"InputLayer mode must be in 0..4, got {mode}")

    def forward(self, input):
        coords, feats = input[0], input[1]
        ops._check_feats(feats)
        if coords.size(1) == self.dimension:  # no batch column: one sample
            coords = torch.cat([coords.long(), torch.zeros_like(coords[:, :1]).long()], 1)
        if coords.size(0) != feats.size(0):
            raise ValueError(f"InputLayer: {coords.size(0)} coordinates but {feats.size(0)} feature rows")
        size = int(self.spatial_size[0])
        meta = take_prefetched(coords, size) if coords.is_cuda else None
        if meta is None:
            meta = Metadata(feats.device)
            meta.build_input(coords.long(), size)
        lvl = meta.level(size)
        self.last_plan = meta.plan
        rules = meta.input
        if self.mode in (3, 4):
            out = ops.InputLayerFunction.apply(feats, rules, lvl.n, self.mode)
        else:
            vs = rules.vstart.long()
            pick = vs[1:] - 1 if self.mode == 1 else vs[:-1]
            out = feats.index_select(0, rules.perm.long().index_select(0, pick))
        return SparseConvNetTensor(out, meta, self.spatial_size)


class OutputLayer(nn.Module):
    """SparseConvNetTensor -> per-point features in the original point order."""

    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension

    def forward(self, input):
        return ops.OutputLayerFunction.apply(input.features, input.metadata.input)


class _ConvBase(nn.Module):
    def __init__(self, dimension, nIn, nOut, filter_size, bias, groups, std_fan_in=True):
        super().__init__()
        _check_dim(dimension)
        if groups != 1:
            raise NotImplementedError("mi3dsparse convolutions implement groups=1")
        self.dimension, self.nIn, self.nOut, self.groups = dimension, nIn, nOut, groups
        self.filter_size = torch.LongTensor([_cube(filter_size, dimension, type(self).__name__)] * dimension)
        self.filter_volume = int(self.filter_size.prod().item())
        std = math.sqrt(2.0 / nIn / self.filter_volume)
        self.weight = nn.Parameter(torch.empty(self.filter_volume, groups, nIn // groups, nOut // groups).normal_(0, std))
        if bias:
            self.bias = nn.Parameter(torch.zeros(nOut))
        else:
            self.bias = None

    def _bias(self, f):
        return f if self.bias is None else f + self.bias


class SubmanifoldConvolution(_ConvBase):
    def __init__(self, dimension, nIn, nOut, filter_size, bias, groups=1):
        super().__init__(dimension, nIn, nOut, filter_size, bias, groups)
        if int(self.filter_size[0]) % 2 != 1:
            raise ValueError("SubmanifoldConvolution needs an odd filter_size")

    def forward(self, input):
        size = input.size_int
        rules = input.metadata.level(size).subm_rules(int(self.filter_size[0]))
        # BatchNorm epilogues (ops.FUSE_BN_STATS): the BN whose output this is gets its backward sums from this
        # convolution's backward-data; a training-mode BN right after it (Sequential sets _bn_next) its forward
        # sums from this forward
        bl = getattr(input, "_bn_link", None)
        link = bl[1] if (bl is not None and bl[0] is input.features) else None
        parts = None
        if self.__dict__.get("_bn_next") and self.bias is None and input.features.is_cuda:
            parts = ops.BnParts(self.nOut, input.features.size(0), input.features.device)
        f = ops.SubmanifoldConvFunction.apply(input.features, self.weight, rules, link, parts)
        f = self._bias(f)
        _count(rules.n_rules * self.nIn * self.nOut, f)
        out = SparseConvNetTensor(f, input.metadata, input.spatial_size)
        if parts is not None and parts.written:
            out._bn_partial = (f, parts)
        return out


class Convolution(_ConvBase):
    def __init__(self, dimension, nIn, nOut, filter_size, filter_stride, bias, groups=1):
        super().__init__(dimension, nIn, nOut, filter_size, bias, groups)
        self.filter_stride = torch.LongTensor([_cube(filter_stride, dimension, "Convolution")] * dimension)
        if int(self.filter_stride[0]) != int(self.filter_size[0]):
            raise NotImplementedError("Convolution: mi3dsparse implements filter_size == filter_stride")

    def forward(self, input):
        stride = int(self.filter_stride[0])
        coarse, rules = input.metadata.downsample(input.size_int, stride)
        parts = None
        if self.__dict__.get("_bn_next") and self.bias is None and input.features.is_cuda:
            parts = ops.BnParts(self.nOut, coarse.n, input.features.device)
        f = ops.ConvolutionFunction.apply(input.features, self.weight, rules, coarse.n, parts)
        f = self._bias(f)
        _count(input.features.size(0) * self.nIn * self.nOut, f)
        size = (input.spatial_size - self.filter_size) // self.filter_stride + 1
        out = SparseConvNetTensor(f, input.metadata, size)
        if parts is not None and parts.written:
            out._bn_partial = (f, parts)
        return out


class Deconvolution(_ConvBase):
    def __init__(self, dimension, nIn, nOut, filter_size, filter_stride, bias, groups=1):
        super().__init__(dimension, nIn, nOut, filter_size, bias, groups)
        self.filter_stride = torch.LongTensor([_cube(filter_stride, dimension, "Deconvolution")] * dimension)
        if int(self.filter_stride[0]) != int(self.filter_size[0]):
            raise NotImplementedError("Deconvolution: mi3dsparse implements filter_size == filter_stride")

    def forward(self, input):
        stride = int(self.filter_stride[0])
        fine, rules = input.metadata.upsample_rules(input.size_int, stride)
        bl = getattr(input, "_bn_link", None)
        link = bl[1] if (bl is not None and bl[0] is input.features) else None
        f = ops.DeconvolutionFunction.apply(input.features, self.weight, rules, fine.n, link)
        f = self._bias(f)
        _count(fine.n * self.nIn * self.nOut, f)
        size = (input.spatial_size - 1) * self.filter_stride + self.filter_size
        return SparseConvNetTensor(f, input.metadata, size)


class NetworkInNetwork(nn.Module):
    """Per-site dense linear map: GEMMs on hipBLASLt via torch, weight gradient
    on msp_conv_wgrad (ops.NetworkInNetworkFunction)."""

    def __init__(self, nIn, nOut, bias=False):
        super().__init__()
        self.nIn, self.nOut = nIn, nOut
        self.weight = nn.Parameter(torch.empty(nIn, nOut).normal_(0, math.sqrt(2.0 / nIn)))
        self.bias = nn.Parameter(torch.zeros(nOut)) if bias else None

    def forward(self, input):
        f = ops.NetworkInNetworkFunction.apply(input.features, self.weight)
        if self.bias is not None:
            f = f + self.bias
        _count(input.features.size(0) * self.nIn * self.nOut, f)
        return SparseConvNetTensor(f, input.metadata, input.spatial_size)


class UnPooling(nn.Module):
    def __init__(self, dimension, pool_size, pool_stride, nFeaturesToDrop=0):
        super().__init__()
        _check_dim(dimension)
        self.dimension = dimension
        self.pool_size = torch.LongTensor([_cube(pool_size, dimension, "UnPooling")] * dimension)
        self.pool_stride = torch.LongTensor([_cube(pool_stride, dimension, "UnPooling")] * dimension)
        if int(self.pool_size[0]) != int(self.pool_stride[0]) or nFeaturesToDrop:
            raise NotImplementedError("UnPooling: pool_size == pool_stride and nFeaturesToDrop == 0 only")

    def forward(self, input):
        stride = int(self.pool_stride[0])
        fine, rules = input.metadata.upsample_rules(input.size_int, stride)
        f = ops.UnPoolingFunction.apply(input.features, rules, fine.n)
        size = (input.spatial_size - 1) * self.pool_stride + self.pool_size
        return SparseConvNetTensor(f, input.metadata, size)


class MaxPooling(nn.Module):
    def __init__(self, dimension, pool_size, pool_stride, nFeaturesToDrop=0):
        super().__init__()
        _check_dim(dimension)
        self.dimension = dimension
        self.pool_size = torch.LongTensor([_cube(pool_size, dimension, "MaxPooling")] * dimension)
        self.pool_stride = torch.LongTensor([_cube(pool_stride, dimension, "MaxPooling")] * dimension)
        if int(self.pool_size[0]) != int(self.pool_stride[0]) or nFeaturesToDrop:
            raise NotImplementedError("MaxPooling: pool_size == pool_stride and nFeaturesToDrop == 0 only")

    def forward(self, input):
        stride = int(self.pool_stride[0])
        coarse, rules = input.metadata.downsample(input.size_int, stride)
        f = ops.MaxPoolingFunction.apply(input.features, rules, coarse.n)
        size = (input.spatial_size - self.pool_size) // self.pool_stride + 1
        return SparseConvNetTensor(f, input.metadata, size)


class BatchNormalization(nn.Module):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9, affine=True, leakiness=1):
        super().__init__()
        self.nPlanes, self.eps, self.momentum, self.affine, self.leakiness = nPlanes, eps, momentum, affine, leakiness
        self.register_buffer("running_mean", torch.zeros(nPlanes))
        self.register_buffer("running_var", torch.ones(nPlanes))
        if affine:
            self.weight = nn.Parameter(torch.ones(nPlanes))
            self.bias = nn.Parameter(torch.zeros(nPlanes))
        else:
            self.weight = self.bias = None

    def forward(self, input):
        if input.features.size(1) != self.nPlanes:
            raise ValueError(f"BatchNormalization({self.nPlanes}) got {input.features.size(1)} channels")
        # a training-mode BN hands its consumer a link: a submanifold convolution's backward-data then leaves
        # this BN's backward sums (ops.BnLink)
        link = ops.BnLink(self.leakiness) if (ops.FUSE_BN_STATS and self.training and input.features.is_cuda) \
            else None
        args = (self.weight, self.bias, self.running_mean, self.running_var, self.eps, self.momentum,
                float(self.leakiness), self.training, self._joined_partial(input), link)
        fork = self.__dict__.pop("_fork", False)
        js = self._join_sources(input)
        if js is not None:
            # x is a JoinTable's [a | b]: the backward writes a's and b's gradients itself, no split pass
            # (ops.BatchNormJoinFunction; with fork, also the shortcut's gradient of x added inside it)
            f, xs = ops.BatchNormJoinFunction.apply(input.features.detach(), js[0], js[1], fork, *args)
            if fork:
                self._fork_shortcut = SparseConvNetTensor(xs, input.metadata, input.spatial_size)
        elif fork:
            # residual fork requested by ConcatTable: x is handed on to the shortcut through the Function so
            # the shortcut's gradient of x is added inside the BN backward (ops.BatchNormForkFunction)
            f, xs = ops.BatchNormForkFunction.apply(input.features, *args)
            self._fork_shortcut = SparseConvNetTensor(xs, input.metadata, input.spatial_size)
        else:
            f = ops.BatchNormFunction.apply(input.features, *args)
        out = SparseConvNetTensor(f, input.metadata, input.spatial_size)
        if link is not None:
            out._bn_link = (f, link)
        return out

    def _join_sources(self, input):
        """(a, b) when input is exactly a two-way JoinTable's output (JoinTable leaves them) and the fused split
        applies (ops.FUSE_JOIN_SPLIT, device tensors, a gradient to propagate)."""
        js = getattr(input, "_join_src", None)
        if js is None or not ops.FUSE_JOIN_SPLIT or js[0] is not input.features or not input.features.is_cuda:
            return None
        a, b = js[1], js[2]
        return (a, b) if (a.requires_grad or b.requires_grad) and torch.is_grad_enabled() else None

    def _joined_partial(self, input):
        """Batch-statistic partials a residual join left on its output (AddTable), if they are for exactly
        these features and this pass needs batch statistics."""
        jp = getattr(input, "_bn_partial", None)
        return jp[1] if (jp is not None and self.training and jp[0] is input.features) else None

    def forward_fork(self, input):
        """(BN-ReLU(input), input) with the shortcut's gradient of input added inside the BN backward.  The
        module is called normally (forward hooks see the usual input and output)."""
        self._fork = True
        try:
            y = self(input)
        finally:
            self.__dict__.pop("_fork", None)
        return y, self.__dict__.pop("_fork_shortcut")

    def extra_repr(self):
        return f"{self.nPlanes}, eps={self.eps}, momentum={self.momentum}, leakiness={self.leakiness}"


class BatchNormReLU(BatchNormalization):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9):
        super().__init__(nPlanes, eps, momentum, True, 0)


class BatchNormLeakyReLU(BatchNormalization):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9, leakiness=0.333):
        super().__init__(nPlanes, eps, momentum, True, leakiness)


# ------------------------------------------------------------------ containers
def _leading_bn(m):
    """The BatchNormalization that consumes a module's input first: m itself, the first child of a Sequential, or
    the BN of a residual fork (ConcatTable(shortcut, Sequential(BN, ...)), which runs its BN first), recursively;
    None otherwise."""
    while True:
        if isinstance(m, Sequential) and len(m) > 0:
            m = m[0]
        elif isinstance(m, ConcatTable) and _fork_bn(list(m._modules.values())) is not None:
            m = _fork_bn(list(m._modules.values()))
        else:
            return m if isinstance(m, BatchNormalization) else None


def _fork_bn(mods):
    """The BN of a residual fork (shortcut, Sequential(BatchNorm, ...)) that ConcatTable runs fused, or None."""
    if FUSE_RESIDUAL and len(mods) == 2 and isinstance(mods[1], nn.Sequential) and len(mods[1]) > 0 \
            and type(mods[1][0]).forward is BatchNormalization.forward:
        return mods[1][0]
    return None


class Sequential(nn.Sequential):
    def add(self, module):
        self._modules[str(len(self._modules))] = module
        return self

    def forward(self, input):
        return _chain(list(self._modules.values()), input)


def _chain(mods, input):
    """Run mods in order (Sequential); a SubmanifoldConvolution followed by a training-mode BatchNorm leaves that
    BN's forward sums in its epilogue (_bn_next, ops.FUSE_BN_STATS)."""
    for i, m in enumerate(mods):
        if ops.FUSE_BN_STATS and type(m) in (SubmanifoldConvolution, Convolution) and i + 1 < len(mods):
            bn = _leading_bn(mods[i + 1])
            if bn is not None and bn.training:
                m._bn_next = True
                try:
                    input = m(input)
                finally:
                    m.__dict__.pop("_bn_next", None)
                continue
        input = m(input)
    return input


# Residual fork / join fusions (ops.BatchNormForkFunction, ops.ResidualJoinFunction); False = SCN's
# one-module-at-a-time composition with torch adds (same results bit for bit, tests/test_gpu_ops.py).
FUSE_RESIDUAL = True


class ConcatTable(nn.Module):
    def __init__(self, *args):
        super().__init__()
        for i, m in enumerate(args):
            self._modules[str(i)] = m

    def add(self, module):
        self._modules[str(len(self._modules))] = module
        return self

    def forward(self, input):
        mods = list(self._modules.values())
        # residual fork (shortcut, Sequential(BatchNorm..., ...)): the BN runs first and hands x on to the
        # shortcut, so x's two gradients are summed inside the BN backward (ops.BatchNormForkFunction)
        if _fork_bn(mods) is not None and input.features.is_cuda:
            y, xs = mods[1][0].forward_fork(input)
            out = mods[0](xs)
            return [out, _chain(list(mods[1])[1:], y)]
        return [m(input) for m in mods]


class AddTable(nn.Module):
    def forward(self, input):
        if FUSE_RESIDUAL and len(input) == 2 and input[0].features.is_cuda and input[0].features.shape == input[1].features.shape:
            # residual join + the next BatchNormalization's statistics in one pass (ops.ResidualJoinFunction)
            f, partial = ops.ResidualJoinFunction.apply(input[0].features, input[1].features)
            out = SparseConvNetTensor(f, input[0].metadata, input[0].spatial_size)
            out._bn_partial = (f, partial)
            return out
        f = input[0].features
        for t in input[1:]:
            f = f + t.features
        return SparseConvNetTensor(f, input[0].metadata, input[0].spatial_size)


class JoinTable(nn.Module):
    """Channel concatenation in branch order on msp_join_cols; in training mode it also
    leaves the batch-statistic partials of its output for the BatchNormalization it feeds (the UNet decoder
    block, the FCN's final BN), like the residual join.  More than two inputs are joined left to right."""

    def forward(self, input):
        f = input[0].features
        partial = None
        if not f.is_cuda:  # the product has no CPU path: fail in the library binding, as every op does
            ops._check_feats(f)
        for k, t in enumerate(input[1:]):
            last = k == len(input) - 2
            f, partial = ops.JoinFunction.apply(f, t.features, bool(FUSE_RESIDUAL and self.training and last))
        out = SparseConvNetTensor(f, input[0].metadata, input[0].spatial_size)
        if partial is not None:
            out._bn_partial = (f, partial)
        if len(input) == 2:  # the BatchNormalization this join feeds may write the inputs' gradients itself
            out._join_src = (f, input[0].features, input[1].features)
        return out


class Identity(nn.Module):
    def forward(self, input):
        return input


class SparseToDense(nn.Module):
    """(B, nPlanes, S, S, S) dense tensor of a sparse tensor (format
    conversion only; Function_test.py:45-53, models/projector/components.py:78-80)."""

    def __init__(self, dimension, nPlanes):
        super().__init__()
        _check_dim(dimension)
        self.dimension, self.nPlanes = dimension, nPlanes

    def forward(self, input):
        S = input.size_int
        loc = input.get_spatial_locations()
        B = input.batch_size()
        f = input.features
        flat = f.new_zeros((B * S * S * S, self.nPlanes))
        idx = ((loc[:, 3] * S + loc[:, 0]) * S + loc[:, 1]) * S + loc[:, 2]
        flat = flat.index_add(0, idx, f)
        return flat.view(B, S, S, S, self.nPlanes).permute(0, 4, 1, 2, 3).contiguous()


def prefetch_metadata(model, coords, wait_for_producer=True):
    """Input pipelining (an addition to the SCN API, optional): build the
    Metadata of the batch with these coords -- voxelisation and every
    rulebook the model's last forward requested -- on a side stream now
    (typically right after the current step's backward/optimizer calls were
    queued), so the next forward on these coords starts with it ready.
    Returns the Metadata, or None before the model's first forward.

    wait_for_producer=True (the safe default) orders the side stream after
    everything already queued on the current stream, in case kernels queued
    there still write `coords`; the build's count reads then wait for the
    queued backward/optimizer too, so there is no overlap.  Pass False for
    coords that are already complete on the device (a resident batch, or one
    whose producer was synchronised): the build then runs beside the queued
    work.  A torch.cuda.Event orders the build after that event only (bench.py
    --graph paces its capture loop this way).  The entry is keyed on the coords
    tensor object itself and only the latest prefetch per device is kept."""
    for m in model.modules():
        if isinstance(m, InputLayer):
            plan = getattr(m, "last_plan", None)
            if plan is None:
                return None
            return prefetch(coords.long(), int(m.spatial_size[0]), list(plan), wait_for_producer)
    return None
