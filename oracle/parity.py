"""Run a device encoder and its oracle twin on the same batch with the same
ReLU decisions -- TEST INFRASTRUCTURE ONLY (see scn_oracle.py header).

Two correct fp32 evaluations of a deep ReLU network can disagree on the sign
of a BatchNorm output that lies within an ulp of zero; the gradient of that
one element then differs by O(|dy|) and the difference spreads backward.  To
compare gradients at fp32 precision the oracle is therefore run with every
BatchNorm-(leaky)ReLU taking the device run's sign decisions (forward values
are still computed independently in fp64).  `flips` reports how many
decisions the oracle would have taken differently, and `max_flip_margin`
the largest |z| among them (it must stay at rounding level).
"""
from __future__ import annotations

import numpy as np
import torch

from . import scn_oracle as O


def raster_perm(loc: np.ndarray, size: int) -> np.ndarray:
    """Permutation taking device rows to the oracle's raster-key row order."""
    key = ((loc[:, 3] * size + loc[:, 0]) * size + loc[:, 1]) * size + loc[:, 2]
    return np.argsort(key, kind="stable")


def run_shared_masks(model, ref, x_dev, x_ref, istrain):
    """Forward both models; returns (out_dev, out_ref, stats)."""
    bn_dev = {n: m for n, m in model.named_modules() if type(m).__name__.startswith("BatchNorm")}
    bn_ref = {n: m for n, m in ref.named_modules() if isinstance(m, O.BatchNormalization)}
    assert bn_dev.keys() == bn_ref.keys()
    caps, hooks = {}, []
    for n, m in bn_dev.items():
        hooks.append(m.register_forward_hook(lambda mod, i, o, n=n: caps.__setitem__(n, o)))
    out_dev = model(x_dev, istrain=istrain)
    for h in hooks:
        h.remove()
    perms = {}
    for n, o in caps.items():
        size = int(o.spatial_size[0])
        if size not in perms:
            loc = o.metadata.locations(size).cpu().numpy()
            perms[size] = torch.from_numpy(raster_perm(loc, size))
        bn_ref[n].forced_mask = (o.features.detach() > 0).cpu()[perms[size]]
    flips, margin = 0, 0.0
    checks = []

    def check(mod, i, o, n):
        x = i[0].features.detach()
        if mod.training:
            mu, var = x.mean(0), x.var(0, unbiased=False)
        else:
            mu, var = mod.running_mean.to(x.dtype), mod.running_var.to(x.dtype)
        z = (x - mu) / torch.sqrt(var + mod.eps) * mod.weight.detach() + mod.bias.detach()
        diff = (z > 0) != mod.forced_mask
        checks.append((int(diff.sum()), float(z[diff].abs().max()) if diff.any() else 0.0))

    for n, m in bn_ref.items():
        hooks.append(m.register_forward_hook(lambda mod, i, o, n=n: check(mod, i, o, n)))
    out_ref = ref(x_ref, istrain=istrain)
    for h in hooks:
        h.remove()
    for m in bn_ref.values():
        m.forced_mask = None
    for f, z in checks:
        flips += f
        margin = max(margin, z)
    return out_dev, out_ref, {"flips": flips, "max_flip_margin": margin}
