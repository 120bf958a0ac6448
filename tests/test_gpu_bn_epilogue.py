"""BatchNorm statistics from convolution epilogues (msp_bn_epilogue).

The submanifold convolution that feeds a training-mode BatchNorm leaves the BN's forward sums (sum v, sum v^2) in
its epilogue, and the backward-data of the convolution a BatchNorm feeds leaves the BN's backward sums (sum dz,
sum dz * xhat).  Per element the arithmetic is the BN statistics passes' own; only the fp64 summation order
differs (per 128-row tile, then tiles in order).  Tolerances, written in each test: the sums against the library's
own statistics passes 1e-12 of the sum of magnitudes (fp64 reordering); the layers and a training step against
the unfused path 1e-5 of each tensor's max (a different fp64 order can move an fp32 statistic by one ulp).
"""
import pytest
import torch

import sparseconvnet as scn
from wsss3d.synthetic import random_cloud

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _level(n=20000, extent=40, seed=0, size=64):
    coords, feats = random_cloud(n, extent, n_batch=2, seed=seed, n_feat=3, dense_frac=0.3)
    t = scn.InputLayer(3, size, mode=4)([torch.from_numpy(coords).to(DEV), torch.from_numpy(feats).to(DEV)])
    lvl = t.metadata.level(size)
    return lvl, lvl.subm_rules(3)


def _bn_stats(xb, leak_seed=0):
    """stats[5][C] of a training-mode BN over xb, from the library's own passes (weight / bias not trivial)."""
    from sparseconvnet import ops
    V, C = xb.shape
    g = torch.Generator().manual_seed(C + leak_seed)
    w = (0.5 + torch.rand(C, generator=g)).to(DEV)
    b = (torch.rand(C, generator=g) - 0.5).to(DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    _, stats = ops._bn_fwd(xb, w, b, rm, rv, 1e-4, 0.9, 0.0, True, None)
    return stats


def _cm_sums(parts):
    C, P = parts.C, parts.P
    return parts.buf[:2 * C * P].view(2, C, P).sum(-1)


@pytest.mark.parametrize("form,cin,cout", [("local", 64, 64), ("local", 96, 64), ("local", 64, 128),
                                           ("tile", 32, 32), ("tile", 64, 32), ("tile", 32, 64)])
@pytest.mark.parametrize("direction,leak", [("fwd", 0.0), ("bwd", 0.0), ("bwd", 0.333)])
def test_conv_epilogue_sums(form, cin, cout, direction, leak):
    """The epilogue's per-tile sums, added over the tiles, equal the library's statistics passes over the rows the
    call wrote (msp_bn_stats forward; msp_bn_bwd_stats with the BN input and stats backward) to fp64 reordering,
    on the tile-local form (64+ channels) and the per-wave tiles (32-channel outputs, and 32 -> 64 in two column
    passes); the output rows are bit-identical to the call without the epilogue."""
    from sparseconvnet import _lib, ops
    # 32 -> 64 takes the per-wave tiles from 10^5 rows (msp_conv_tile_form)
    lvl, rules = _level(300000, 120, cin + cout, 128) if (cin, cout) == (32, 64) else _level(seed=cin + cout)
    V = lvl.n
    assert V >= 4096
    torch.manual_seed(cin * 3 + cout)
    x = torch.randn(V, cin, device=DEV)
    w = torch.randn(27, cin, cout, device=DEV) / (27 * cin) ** 0.5
    f = ops.conv_form(rules, V, cin, cout, 27)
    assert (f == "local") == (form == "local")
    assert ops.bn_epi_ok(rules, V, cin, cout, 27)
    parts = ops.BnParts(cout, V, x.device)
    if direction == "fwd":
        epi = (parts, None, None, 0.0)
        xb = stats = None
    else:
        xb = torch.randn(V, cout, device=DEV) * 1.5 + 0.3
        stats = _bn_stats(xb)
        epi = (parts, xb, stats, leak)
    y = ops.conv_tile(x, w, 27, 2, cout, rules, V, epi=epi)
    y0 = ops.conv_tile(x, w, 27, 2, cout, rules, V)
    assert parts.written and torch.equal(y, y0)
    got = _cm_sums(parts)
    ref_part = ops._bn_partial_buf(V, cout, x.device)
    if direction == "fwd":
        _lib.call("msp_bn_stats", _lib.ptr(y), V, cout, _lib.ptr(ref_part), ops._stream(y))
        mag = torch.stack([y.double().abs().sum(0), y.double().square().sum(0)])
    else:
        _lib.call("msp_bn_bwd_stats", _lib.ptr(xb), _lib.ptr(y), V, cout, _lib.ptr(stats), float(leak),
                  _lib.ptr(ref_part), ops._stream(y))
        mag = torch.stack([y.double().abs().sum(0), (y.double() * xb.double()).abs().sum(0) * 10])
    Pr = int(_lib.query("msp_bn_partials", _lib.I64(V), cout))
    ref = ref_part[:Pr * 2 * cout].view(Pr, 2, cout).sum(0)
    err = ((got - ref).abs() / mag.clamp_min(1e-30)).max().item()
    print(f"{form} {cin}->{cout} {direction} leak {leak}: V={V} P={parts.P} max rel err {err:.2e}")
    assert err < 1e-12, err


def _unet_step(fuse, monkeypatch, m=32, reps=2, seed=5):
    from sparseconvnet import ops
    from wsss3d import EasyDict, MODEL_REGISTRY
    from wsss3d.synthetic import make_batch
    monkeypatch.setattr(ops, "FUSE_BN_STATS", fuse)
    counts = {}
    real_call = ops.call

    def counting(name, *a):
        counts[name] = counts.get(name, 0) + 1
        return real_call(name, *a)
    monkeypatch.setattr(ops, "call", counting)
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("SparseConvUNet")
    model = cls("SparseConvUNet", m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=True).to(DEV)
    b = make_batch(2, 50, seed=seed)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                 batch_offsets=b["batch_offsets"])
    out = model(x)
    wgt = torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)
    (out * wgt).sum().backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    bufs = {n: t.detach().clone() for n, t in model.named_buffers()}
    monkeypatch.setattr(ops, "call", real_call)
    return out.detach(), grads, bufs, counts


def test_training_step_fused_matches_unfused(monkeypatch):
    """The headline network (SparseConvUNet m=32, reps 2, residual) on two scenes at 2 cm, one forward + backward
    with the BatchNorm epilogues against the same step with every BN running its own statistics passes: scene
    features, every parameter gradient and the running statistics within 1e-5 of each tensor's max (the fp64 sums
    are only reordered).  The fused step must run the epilogues on both forms (tile-local at levels 1-4, per-wave
    tiles at level 0) in both directions, and skip that many statistics passes."""
    out1, g1, b1, c1 = _unet_step(True, monkeypatch)
    out0, g0, b0, c0 = _unet_step(False, monkeypatch)
    print({k: (c1.get(k, 0), c0.get(k, 0)) for k in sorted(set(c1) | set(c0)) if "bn" in k or "conv" in k})
    for name in ("msp_conv_local_bn", "msp_conv_tile_bn", "msp_bn_finalize_cm", "msp_bn_bwd_apply_cm"):
        assert c1.get(name, 0) > 0 and c0.get(name, 0) == 0, name
    # every forward sum the epilogue left replaces one statistics pass, every backward sum one backward pass
    assert c0.get("msp_bn_stats", 0) - c1.get("msp_bn_stats", 0) == c1["msp_bn_finalize_cm"]
    assert c0["msp_bn_bwd_stats"] - c1.get("msp_bn_bwd_stats", 0) == c1["msp_bn_bwd_apply_cm"]

    def rel(a, b):
        return (a.double() - b.double()).abs().max().item() / max(b.double().abs().max().item(), 1e-30)
    assert rel(out1, out0) < 1e-5, rel(out1, out0)
    worst = max(rel(g1[n], g0[n]) for n in g0)
    assert worst < 1e-5, worst
    for n in b0:
        assert rel(b1[n], b0[n]) < 1e-5, n


def test_epilogue_skipped_when_gradient_is_not_the_convolutions(monkeypatch):
    """A BN whose output has a second consumer gets the sum of two gradients, not the tensor the convolution's
    backward-data returned: it must run its own statistics pass (the link is checked by identity), and the
    gradients equal the unfused path's to fp64 reordering."""
    from sparseconvnet import ops
    from sparseconvnet.sparseConvNetTensor import SparseConvNetTensor
    coords, feats = random_cloud(20000, 40, n_batch=2, seed=7, n_feat=3, dense_frac=0.3)
    t = scn.InputLayer(3, 64, mode=4)([torch.from_numpy(coords).to(DEV), torch.from_numpy(feats).to(DEV)])
    V = t.features.size(0)
    results = []
    for fuse in (True, False):
        monkeypatch.setattr(ops, "FUSE_BN_STATS", fuse)
        counts = {}
        real_call = ops.call

        def counting(name, *a):
            counts[name] = counts.get(name, 0) + 1
            return real_call(name, *a)
        monkeypatch.setattr(ops, "call", counting)
        torch.manual_seed(3)
        bn = scn.BatchNormReLU(64).to(DEV)
        conv = scn.SubmanifoldConvolution(3, 64, 64, 3, False).to(DEV)
        x = (torch.randn(V, 64, device=DEV) * 2 + 0.5).requires_grad_(True)
        y = bn(SparseConvNetTensor(x, t.metadata, t.spatial_size))
        z = conv(y)
        wz = torch.linspace(-1, 1, z.features.numel(), device=DEV).view_as(z.features)
        ((z.features * wz).sum() + (y.features * 0.5).sum()).backward()  # y has a second consumer
        monkeypatch.setattr(ops, "call", real_call)
        # the convolution left its sums (the form has the epilogue) but the BN did not take them
        assert counts.get("msp_conv_local_bn", 0) == (1 if fuse else 0)
        assert counts.get("msp_bn_bwd_apply_cm", 0) == 0 and counts.get("msp_bn_bwd_stats", 0) == 1
        results.append((x.grad.clone(), bn.weight.grad.clone(), conv.weight.grad.clone()))
    for a, b in zip(*results):
        assert torch.equal(a, b)
