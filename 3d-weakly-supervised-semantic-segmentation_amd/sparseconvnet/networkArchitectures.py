"""UNet / FullyConvolutionalNet builders.

Topology as used by `models/SparseConvNet.py:63-68,79-85` and restated in the
reference at `Function_test.py:113-164` (UNet encoder half) and
`:166-226` (FCN).  The module tree (and so every state_dict key) follows
SCN's builders: per level `reps` blocks, then a ConcatTable(Identity,
Sequential(BN, Convolution, <next level>, [BN, Deconvolution] | [UnPooling]))
and a JoinTable; the UNet adds `reps` decoder blocks after the join, the
first of them taking the 2x-wide joined input (NetworkInNetwork shortcut when
residual).
"""
from __future__ import annotations

from .modules import (AddTable, BatchNormLeakyReLU, BatchNormReLU, ConcatTable, Convolution, Deconvolution,
                      Identity, JoinTable, NetworkInNetwork, Sequential, SubmanifoldConvolution, UnPooling)


def _block(seq, dimension, a, b, residual, norm):
    """Append one VGG block (norm, SubM a->b) or one residual block
    (ConcatTable(shortcut, norm-SubM-norm-SubM) + AddTable) to `seq`."""
    if residual:
        # shortcut first: parameters are created (and drawn from the RNG) in
        # the same order as SCN's builder, so a seeded init matches it
        shortcut = Identity() if a == b else NetworkInNetwork(a, b, False)
        branch = Sequential()
        branch.add(norm(a)).add(SubmanifoldConvolution(dimension, a, b, 3, False))
        branch.add(norm(b)).add(SubmanifoldConvolution(dimension, b, b, 3, False))
        seq.add(ConcatTable().add(shortcut).add(branch)).add(AddTable())
    else:
        seq.add(Sequential().add(norm(a)).add(SubmanifoldConvolution(dimension, a, b, 3, False)))


def UNet(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2], leakiness=0, n_input_planes=-1):
    def norm(c):
        return BatchNormLeakyReLU(c, leakiness=leakiness)

    def level(planes, n_in):
        seq = Sequential()
        for _ in range(reps):
            _block(seq, dimension, n_in if n_in != -1 else planes[0], planes[0], residual_blocks, norm)
            n_in = -1
        if len(planes) > 1:
            down = Sequential()
            down.add(norm(planes[0]))
            down.add(Convolution(dimension, planes[0], planes[1], downsample[0], downsample[1], False))
            down.add(level(planes[1:], -1))
            down.add(norm(planes[1]))
            down.add(Deconvolution(dimension, planes[1], planes[0], downsample[0], downsample[1], False))
            seq.add(ConcatTable().add(Identity()).add(down))
            seq.add(JoinTable())
            for i in range(reps):
                _block(seq, dimension, planes[0] * (2 if i == 0 else 1), planes[0], residual_blocks, norm)
        return seq

    return level(list(nPlanes), n_input_planes)


def FullyConvolutionalNet(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2]):
    """Output channels = sum(nPlanes): every level upsampled back (UnPooling)
    and joined (models/SparseConvNet.py:73,86)."""

    def level(planes):
        seq = Sequential()
        for _ in range(reps):
            _block(seq, dimension, planes[0], planes[0], residual_blocks, BatchNormReLU)
        if len(planes) > 1:
            down = Sequential()
            down.add(BatchNormReLU(planes[0]))
            down.add(Convolution(dimension, planes[0], planes[1], downsample[0], downsample[1], False))
            down.add(level(planes[1:]))
            down.add(UnPooling(dimension, downsample[0], downsample[1]))
            seq.add(ConcatTable().add(Identity()).add(down))
            seq.add(JoinTable())
        return seq

    return level(list(nPlanes))


def FullyConvolutionalNetEncoder(dimension, reps, nPlanes, residual_blocks=False, downsample=[2, 2]):
    """FCN without the skip joins: each level hands its deepest features back
    up through UnPooling, so the output has nPlanes[-1] channels
    (Function_test.py:166-226; the shape of the reference's unregistered
    `SparseConvFCNetEncoder`, README.md:28, and of the in-repo `FCNEncoder`,
    models/SparseConvNet.py:110-143)."""

    def level(planes):
        seq = Sequential()
        for _ in range(reps):
            _block(seq, dimension, planes[0], planes[0], residual_blocks, BatchNormReLU)
        if len(planes) > 1:
            down = Sequential()
            down.add(BatchNormReLU(planes[0]))
            down.add(Convolution(dimension, planes[0], planes[1], downsample[0], downsample[1], False))
            down.add(level(planes[1:]))
            down.add(UnPooling(dimension, downsample[0], downsample[1]))
            seq.add(down)
        return seq

    return level(list(nPlanes))
