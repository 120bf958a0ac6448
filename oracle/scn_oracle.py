"""CPU ORACLE for the sparse-conv hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product (libmi3dsparse + the `sparseconvnet` package) never calls it.

What it restates: SparseConvNet 0.2's CPU semantics for the `scn.*` surface
that the reference uses (models/SparseConvNet.py:57-229; Function_test.py:35-
232).  SCN itself is a third-party dependency pinned as
`sparseconvnet 0.2 dev` (requirements.txt:2, env_list.txt:246) that is not
vendored under /root/reference and cannot be installed offline, so its
published algorithm is restated here from its documented behaviour:

  * host hash of integer voxel keys per InputLayer call (here: raster keys
    ((b*S + x)*S + y)*S + z, np.unique), mode 4 = average, mode 3 = sum;
  * submanifold rulebook: for every active site and every offset of the f^3
    box (last axis fastest) the (neighbour, site) pair if the neighbour is
    active; forward = per-offset gather -> mm -> scatter-add (SCN's CPU
    backend structure);
  * size==stride Convolution: parent = floor(x / s), offset = position in the
    s^3 block; Deconvolution = its transpose on the same rules; UnPooling
    copies the parent row; MaxPooling takes the max over children;
  * BatchNormalization(eps=1e-4, momentum=0.9, leakiness): batch mean and
    biased variance in train mode, running = m*running + (1-m)*batch with the
    unbiased variance, (leaky) ReLU after the affine;
  * NetworkInNetwork = x @ W; JoinTable concatenates in branch order.

Gradients come from torch autograd over these ops (index_select / mm /
index_add), i.e. the exact adjoint of the forward.  With LEAN = True (the
default) the submanifold convolution and the BatchNormalization run as
autograd Functions with hand-written adjoints that save only their inputs and
recompute the per-offset gathers in backward -- the same arithmetic, but the
8-scene headline batch's fp64 backward then fits in host memory (autograd
saved every gathered (rules x C) matrix and every BN intermediate);
tests/test_oracle.py checks the two forms against each other.  Any float dtype
works: float64 for golden fixtures, float32 for the CPU baseline.

Parity status: "parity unpinned" against SCN itself -- the reference ships no
SCN fixtures or tests.  The oracle is pinned instead by
(1) torch's dense conv3d / conv_transpose3d on small grids
(tests/test_oracle.py), (2) the reference's own encoder definitions
(models/SparseConvNet.py loaded unmodified on top of this module,
tests/golden/make_golden.py) and (3) hand-worked known answers.
"""
from __future__ import annotations

import math
import sys

import numpy as np
import torch
from torch import nn

forward_pass_multiplyAdd_count = 0
forward_pass_hidden_states = 0
LEAN = True  # hand-written adjoints for SubmanifoldConvolution / BatchNormalization (see the header)


def _count(macs, f):
    mod = sys.modules[__name__]
    mod.forward_pass_multiplyAdd_count += int(macs)
    mod.forward_pass_hidden_states += int(f.nelement())


def _int(v):
    if torch.is_tensor(v):
        v = v.view(-1)[0].item()
    elif isinstance(v, (list, tuple)):
        v = v[0]
    return int(v)


class OLevel:
    def __init__(self, size, coords):
        self.size = size
        self.coords = coords  # (V, 4) int64 numpy [x, y, z, b], sorted by raster key
        S = size
        self.keys = ((coords[:, 3] * S + coords[:, 0]) * S + coords[:, 1]) * S + coords[:, 2]
        self.subm = {}
        self.down = {}

    @property
    def n(self):
        return len(self.keys)

    def lookup(self, c):
        """Row index of each coordinate row in c (or -1)."""
        S = self.size
        ok = np.all((c[:, :3] >= 0) & (c[:, :3] < S), axis=1)
        k = ((c[:, 3] * S + c[:, 0]) * S + c[:, 1]) * S + c[:, 2]
        pos = np.searchsorted(self.keys, k)
        pos = np.minimum(pos, max(self.n - 1, 0))
        hit = ok & (self.n > 0) & (self.keys[pos] == k) if self.n else np.zeros(len(c), bool)
        return np.where(hit, pos, -1)

    def subm_rules(self, f):
        """list over offsets of (in_idx, out_idx) int64 numpy arrays."""
        if f not in self.subm:
            h = f // 2
            rules = []
            for dx in range(-h, h + 1):
                for dy in range(-h, h + 1):
                    for dz in range(-h, h + 1):
                        nb = self.coords + np.array([dx, dy, dz, 0])
                        idx = self.lookup(nb)
                        out = np.nonzero(idx >= 0)[0]
                        rules.append((idx[out], out))
            self.subm[f] = rules
        return self.subm[f]


class OMeta:
    def __init__(self):
        self.levels = {}
        self.p2v = None
        self.counts = None
        self.n_points = 0

    def downsample(self, size, s):
        key = (size, s)
        if key not in self.levels[size].down:
            fine = self.levels[size]
            pc = fine.coords.copy()
            pc[:, :3] //= s
            csize = size // s
            ck = ((pc[:, 3] * csize + pc[:, 0]) * csize + pc[:, 1]) * csize + pc[:, 2]
            uk, first, parent = np.unique(ck, return_index=True, return_inverse=True)
            coarse = self.levels.get(csize)
            if coarse is None:
                coarse = OLevel(csize, pc[first])
                self.levels[csize] = coarse
            loc = fine.coords[:, :3] % s
            offset = (loc[:, 0] * s + loc[:, 1]) * s + loc[:, 2]
            self.levels[size].down[key] = (csize, parent.reshape(-1), offset)
        return self.levels[size].down[key]


class OTensor:
    def __init__(self, features, metadata, spatial_size):
        self.features, self.metadata = features, metadata
        self.spatial_size = torch.LongTensor([int(spatial_size)] * 3)

    @property
    def size(self):
        return int(self.spatial_size[0])


class InputLayer(nn.Module):
    def __init__(self, dimension, spatial_size, mode=3):
        super().__init__()
        self.size, self.mode = _int(spatial_size), mode

    def forward(self, input):
        coords = input[0].detach().cpu().long().numpy()
        feats = input[1]
        if coords.shape[1] == 3:
            coords = np.concatenate([coords, np.zeros((len(coords), 1), np.int64)], 1)
        S = self.size
        keys = ((coords[:, 3] * S + coords[:, 0]) * S + coords[:, 1]) * S + coords[:, 2]
        uk, first, inv = np.unique(keys, return_index=True, return_inverse=True)
        inv = inv.reshape(-1)
        meta = OMeta()
        meta.levels[S] = OLevel(S, coords[first])
        meta.p2v = torch.from_numpy(inv)
        meta.n_points = len(coords)
        cnt = torch.from_numpy(np.bincount(inv, minlength=len(uk))).to(feats.dtype)
        meta.counts = cnt
        out = feats.new_zeros((len(uk), feats.size(1))).index_add(0, meta.p2v, feats)
        if self.mode == 4:
            out = out / cnt[:, None]
        elif self.mode != 3:
            raise NotImplementedError("oracle implements InputLayer modes 3 and 4")
        return OTensor(out, meta, S)


class OutputLayer(nn.Module):
    def __init__(self, dimension):
        super().__init__()

    def forward(self, input):
        return input.features.index_select(0, input.metadata.p2v)


class SubmanifoldConvolution(nn.Module):
    def __init__(self, dimension, nIn, nOut, filter_size, bias, groups=1):
        super().__init__()
        self.f = _int(filter_size)
        fv = self.f ** 3
        self.nIn, self.nOut = nIn, nOut
        self.weight = nn.Parameter(torch.empty(fv, 1, nIn, nOut).normal_(0, math.sqrt(2.0 / nIn / fv)))
        self.bias = nn.Parameter(torch.zeros(nOut)) if bias else None

    def forward(self, input):
        x = input.features
        rules = input.metadata.levels[input.size].subm_rules(self.f)
        W = self.weight[:, 0]
        nr = sum(len(i_in) for i_in, _ in rules)
        if LEAN:
            out = _SubmConvFn.apply(x, W, rules)
        else:
            out = x.new_zeros((x.size(0), self.nOut))
            for o, (i_in, i_out) in enumerate(rules):
                if len(i_in) == 0:
                    continue
                ii, io = torch.from_numpy(i_in), torch.from_numpy(i_out)
                out = out.index_add(0, io, x.index_select(0, ii) @ W[o])
        if self.bias is not None:
            out = out + self.bias
        _count(nr * self.nIn * self.nOut, out)
        return OTensor(out, input.metadata, input.size)


class _SubmConvFn(torch.autograd.Function):
    """out[i_out] += x[i_in] @ W[o] per offset (the loop above); backward recomputes each offset's gather:
    dx[i_in] += g[i_out] @ W[o]^T, dW[o] = x[i_in]^T @ g[i_out] -- the adjoint autograd derives, without saving
    the gathered matrices."""

    @staticmethod
    def forward(ctx, x, W, rules):
        out = x.new_zeros((x.size(0), W.size(2)))
        idx = []
        for i_in, i_out in rules:
            ii, io = torch.from_numpy(i_in), torch.from_numpy(i_out)
            idx.append((ii, io))
            if len(i_in):
                out.index_add_(0, io, x.index_select(0, ii) @ W[len(idx) - 1])
        ctx.save_for_backward(x, W)
        ctx.idx = idx
        return out

    @staticmethod
    def backward(ctx, g):
        x, W = ctx.saved_tensors
        dx = torch.zeros_like(x) if ctx.needs_input_grad[0] else None
        dW = torch.zeros_like(W) if ctx.needs_input_grad[1] else None
        for o, (ii, io) in enumerate(ctx.idx):
            if len(ii) == 0:
                continue
            go = g.index_select(0, io)
            if dx is not None:
                dx.index_add_(0, ii, go @ W[o].t())
            if dW is not None:
                dW[o] = x.index_select(0, ii).t() @ go
        return dx, dW, None


class Convolution(nn.Module):
    def __init__(self, dimension, nIn, nOut, filter_size, filter_stride, bias, groups=1):
        super().__init__()
        self.s = _int(filter_size)
        assert self.s == _int(filter_stride)
        fv = self.s ** 3
        self.nIn, self.nOut = nIn, nOut
        self.weight = nn.Parameter(torch.empty(fv, 1, nIn, nOut).normal_(0, math.sqrt(2.0 / nIn / fv)))
        self.bias = nn.Parameter(torch.zeros(nOut)) if bias else None

    def forward(self, input):
        x = input.features
        csize, parent, offset = input.metadata.downsample(input.size, self.s)
        Vc = input.metadata.levels[csize].n
        W = self.weight[:, 0]
        out = x.new_zeros((Vc, self.nOut))
        for o in range(W.size(0)):
            sel = np.nonzero(offset == o)[0]
            if len(sel):
                out = out.index_add(0, torch.from_numpy(parent[sel]), x.index_select(0, torch.from_numpy(sel)) @ W[o])
        if self.bias is not None:
            out = out + self.bias
        _count(x.size(0) * self.nIn * self.nOut, out)
        return OTensor(out, input.metadata, csize)


class Deconvolution(nn.Module):
    def __init__(self, dimension, nIn, nOut, filter_size, filter_stride, bias, groups=1):
        super().__init__()
        self.s = _int(filter_size)
        fv = self.s ** 3
        self.nIn, self.nOut = nIn, nOut
        self.weight = nn.Parameter(torch.empty(fv, 1, nIn, nOut).normal_(0, math.sqrt(2.0 / nIn / fv)))
        self.bias = nn.Parameter(torch.zeros(nOut)) if bias else None

    def forward(self, input):
        x = input.features
        fsize = input.size * self.s
        _, parent, offset = input.metadata.downsample(fsize, self.s)
        W = self.weight[:, 0]
        out = x.new_zeros((len(parent), self.nOut))
        for o in range(W.size(0)):
            sel = np.nonzero(offset == o)[0]
            if len(sel):
                out = out.index_add(0, torch.from_numpy(sel), x.index_select(0, torch.from_numpy(parent[sel])) @ W[o])
        if self.bias is not None:
            out = out + self.bias
        _count(len(parent) * self.nIn * self.nOut, out)
        return OTensor(out, input.metadata, fsize)


class UnPooling(nn.Module):
    def __init__(self, dimension, pool_size, pool_stride, nFeaturesToDrop=0):
        super().__init__()
        self.s = _int(pool_stride)

    def forward(self, input):
        fsize = input.size * self.s
        _, parent, _ = input.metadata.downsample(fsize, self.s)
        return OTensor(input.features.index_select(0, torch.from_numpy(parent)), input.metadata, fsize)


class MaxPooling(nn.Module):
    def __init__(self, dimension, pool_size, pool_stride, nFeaturesToDrop=0):
        super().__init__()
        self.s = _int(pool_stride)

    def forward(self, input):
        x = input.features
        csize, parent, _ = input.metadata.downsample(input.size, self.s)
        Vc = input.metadata.levels[csize].n
        idx = torch.from_numpy(parent)[:, None].expand(-1, x.size(1))
        out = x.new_full((Vc, x.size(1)), -float("inf")).scatter_reduce(0, idx, x, "amax", include_self=False)
        return OTensor(out, input.metadata, csize)


class BatchNormalization(nn.Module):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9, affine=True, leakiness=1):
        super().__init__()
        self.eps, self.momentum, self.leak = eps, momentum, leakiness
        self.register_buffer("running_mean", torch.zeros(nPlanes))
        self.register_buffer("running_var", torch.ones(nPlanes))
        self.weight = nn.Parameter(torch.ones(nPlanes)) if affine else None
        self.bias = nn.Parameter(torch.zeros(nPlanes)) if affine else None
        # Optional (V, C) bool mask of the (leaky) ReLU's positive side, set by
        # oracle/parity.py to the device run's decisions: a ReLU input within
        # an ulp of 0 can land on either side in two valid fp32 evaluations,
        # and the gradient of that element then differs by O(|dy|).
        self.forced_mask = None

    def forward(self, input):
        x = input.features
        if self.training:
            mean = x.mean(0)
            var = x.var(0, unbiased=False)
            n = x.size(0)
            with torch.no_grad():
                unb = var * n / max(n - 1, 1)
                self.running_mean.mul_(self.momentum).add_((1 - self.momentum) * mean.detach().to(self.running_mean))
                self.running_var.mul_(self.momentum).add_((1 - self.momentum) * unb.detach().to(self.running_var))
        else:
            mean = self.running_mean.to(x.dtype)
            var = self.running_var.to(x.dtype)
        if LEAN and self.weight is not None:
            y = _BNReLUFn.apply(x, self.weight, self.bias, mean.detach(), var.detach(), self.eps, self.leak,
                                self.training, self.forced_mask)
            return OTensor(y, input.metadata, input.size)
        y = (x - mean) / torch.sqrt(var + self.eps)
        if self.weight is not None:
            y = y * self.weight + self.bias
        pos = (y > 0) if self.forced_mask is None else self.forced_mask
        y = torch.where(pos, y, y * self.leak)
        return OTensor(y, input.metadata, input.size)


class _BNReLUFn(torch.autograd.Function):
    """y = (leaky) ReLU(xhat * w + b), xhat = (x - mean) / sqrt(var + eps), with the batch statistics' own gradient
    in train mode (mean and var are functions of x): the adjoint autograd derives for the composition above,
    written out so that only x is saved:
      dz = dy (z > 0, or the forced mask) else leak dy;  db = sum dz;  dw = sum dz xhat
      train: dx = w invstd (dz - mean(dz) - xhat mean(dz xhat));  eval: dx = w invstd dz"""

    @staticmethod
    def forward(ctx, x, w, b, mean, var, eps, leak, train, mask):
        invstd = 1.0 / torch.sqrt(var + eps)
        z = (x - mean) * invstd * w + b
        pos = (z > 0) if mask is None else mask
        ctx.save_for_backward(x, w, mean, invstd, pos)
        ctx.leak, ctx.train = leak, train
        return torch.where(pos, z, z * leak)

    @staticmethod
    def backward(ctx, gy):
        x, w, mean, invstd, pos = ctx.saved_tensors
        xh = (x - mean) * invstd
        dz = torch.where(pos, gy, gy * ctx.leak)
        db, dw = dz.sum(0), (dz * xh).sum(0)
        if ctx.train:
            dx = w * invstd * (dz - dz.mean(0) - xh * (dz * xh).mean(0))
        else:
            dx = w * invstd * dz
        return dx, dw, db, None, None, None, None, None, None


class BatchNormReLU(BatchNormalization):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9):
        super().__init__(nPlanes, eps, momentum, True, 0)


class BatchNormLeakyReLU(BatchNormalization):
    def __init__(self, nPlanes, eps=1e-4, momentum=0.9, leakiness=0.333):
        super().__init__(nPlanes, eps, momentum, True, leakiness)


class NetworkInNetwork(nn.Module):
    def __init__(self, nIn, nOut, bias=False):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(nIn, nOut).normal_(0, math.sqrt(2.0 / nIn)))
        self.bias = nn.Parameter(torch.zeros(nOut)) if bias else None

    def forward(self, input):
        f = input.features @ self.weight
        if self.bias is not None:
            f = f + self.bias
        _count(input.features.size(0) * self.weight.size(0) * self.weight.size(1), f)
        return OTensor(f, input.metadata, input.size)


class Sequential(nn.Sequential):
    def add(self, module):
        self._modules[str(len(self._modules))] = module
        return self


class ConcatTable(nn.Module):
    def __init__(self, *args):
        super().__init__()
        for i, m in enumerate(args):
            self._modules[str(i)] = m

    def add(self, module):
        self._modules[str(len(self._modules))] = module
        return self

    def forward(self, input):
        return [m(input) for m in self._modules.values()]


class AddTable(nn.Module):
    def forward(self, input):
        return OTensor(sum(t.features for t in input), input[0].metadata, input[0].size)


class JoinTable(nn.Module):
    def forward(self, input):
        return OTensor(torch.cat([t.features for t in input], 1), input[0].metadata, input[0].size)


class Identity(nn.Module):
    def forward(self, input):
        return input


def _vgg_or_residual(m, a, b, residual, bn):
    if residual:
        m.add(ConcatTable()
              .add(Identity() if a == b else NetworkInNetwork(a, b, False))
              .add(Sequential().add(bn(a)).add(SubmanifoldConvolution(3, a, b, 3, False))
                   .add(bn(b)).add(SubmanifoldConvolution(3, b, b, 3, False)))).add(AddTable())
    else:
        m.add(Sequential().add(bn(a)).add(SubmanifoldConvolution(3, a, b, 3, False)))


def UNet(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2], leakiness=0, n_input_planes=-1):
    """SCN UNet: encoder half as Function_test.py:113-164 plus BN+Deconvolution
    on the way up, JoinTable, decoder blocks."""
    bn = lambda c: BatchNormLeakyReLU(c, leakiness=leakiness)  # noqa: E731

    def U(planes, n_in=-1):
        m = Sequential()
        for _ in range(reps):
            _vgg_or_residual(m, n_in if n_in != -1 else planes[0], planes[0], residual_blocks, bn)
            n_in = -1
        if len(planes) > 1:
            m.add(ConcatTable().add(Identity()).add(
                Sequential().add(bn(planes[0])).add(Convolution(3, planes[0], planes[1], downsample[0], downsample[1], False))
                .add(U(planes[1:])).add(bn(planes[1]))
                .add(Deconvolution(3, planes[1], planes[0], downsample[0], downsample[1], False))))
            m.add(JoinTable())
            for i in range(reps):
                _vgg_or_residual(m, planes[0] * (2 if i == 0 else 1), planes[0], residual_blocks, bn)
        return m

    return U(list(nPlanes), n_input_planes)


def FullyConvolutionalNet(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2]):
    def U(planes):
        m = Sequential()
        for _ in range(reps):
            _vgg_or_residual(m, planes[0], planes[0], residual_blocks, BatchNormReLU)
        if len(planes) > 1:
            m.add(ConcatTable().add(Identity()).add(
                Sequential().add(BatchNormReLU(planes[0]))
                .add(Convolution(3, planes[0], planes[1], downsample[0], downsample[1], False))
                .add(U(planes[1:])).add(UnPooling(3, downsample[0], downsample[1]))))
            m.add(JoinTable())
        return m

    return U(list(nPlanes))


def FullyConvolutionalNetEncoder(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2]):
    """Function_test.py:166-226."""
    def U(planes):
        m = Sequential()
        for _ in range(reps):
            _vgg_or_residual(m, planes[0], planes[0], residual_blocks, BatchNormReLU)
        if len(planes) > 1:
            m.add(Sequential().add(BatchNormReLU(planes[0]))
                  .add(Convolution(3, planes[0], planes[1], downsample[0], downsample[1], False))
                  .add(U(planes[1:])).add(UnPooling(3, downsample[0], downsample[1])))
        return m

    return U(list(nPlanes))


def is_power2(n):
    return n != 0 and (n & (n - 1)) == 0


SparseConvNetTensor = OTensor
