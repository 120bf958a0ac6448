"""Oracle encoders -- TEST INFRASTRUCTURE ONLY (see scn_oracle.py header).

Restates the reference's registered encoders (models/SparseConvNet.py:57-229)
on top of the CPU oracle ops, with the same module tree as the product so a
state_dict moves between the two unchanged.  tests/golden/make_golden.py
checks, in the container where /root/reference exists, that these trees match
the reference file's own getEncoder() code driven by the same oracle.
"""
from __future__ import annotations

import torch
from torch import nn

from . import scn_oracle as O

EMBED = {
    "SparseConvUNet": lambda m: m,                               # :57
    "SparseConvFCNet": lambda m: 7 * 8 * m // 2,                 # :73
    "SparseConvFCNetNarrow": lambda m: m + 64 + 128 + 192 + 256,  # :90
    "SparseConvFCNetDirectUpPool": lambda m: 256,                # :107
    "SparseConvFCNetDirectUpPoolLight": lambda m: 128,           # :160
    "SparseConvFCNetEncoder": lambda m: 7 * m,                   # README.md:28, Function_test.py:228-232
}


def _body(name, m, reps, residual):
    lv = [(i + 1) * m for i in range(7)]
    if name == "SparseConvUNet":
        return O.UNet(3, reps, lv, residual), m
    if name == "SparseConvFCNet":
        return O.FullyConvolutionalNet(3, reps, lv, residual), sum(lv)
    if name == "SparseConvFCNetNarrow":
        p = [m, 64, 128, 192, 256]
        return O.FullyConvolutionalNet(3, reps, p, residual), sum(p)
    if name == "SparseConvFCNetDirectUpPool":
        return O.FullyConvolutionalNetEncoder(3, reps, [m, 64, 128, 192, 256], residual), 256
    if name == "SparseConvFCNetDirectUpPoolLight":
        return O.FullyConvolutionalNetEncoder(3, reps, [m, 32, 64, 96, 128], residual, [4, 4]), 128
    if name == "SparseConvFCNetEncoder":
        return O.FullyConvolutionalNetEncoder(3, reps, lv, residual), 7 * m
    raise KeyError(name)


class OracleEncoder(nn.Module):
    def __init__(self, name, m, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False):
        super().__init__()
        inp = O.InputLayer(3, full_scale, mode=4)
        first = O.SubmanifoldConvolution(3, 3, m, 3, False)  # created before the body, as the reference does
        body, out = _body(name, m, block_reps, residual_blocks)
        self.encoder = O.Sequential(inp, first, body, O.BatchNormReLU(out), O.OutputLayer(3))

    def forward(self, x, istrain=False):
        out = self.encoder([x["coords"], x["feature"]])
        if istrain:
            off = list(x["batch_offsets"])
            out = torch.stack([out[off[b]:off[b + 1]].mean(0) for b in range(len(off) - 1)])
        return out
