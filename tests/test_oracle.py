"""Pin the CPU oracle (no GPU needed).

SCN is not available, so the oracle's restatement of each op is checked
against an independent implementation -- torch's dense conv3d /
conv_transpose3d / max_pool3d / batch_norm on the same voxels -- against
hand-worked answers, and against the committed fixtures
(tests/golden/make_golden.py).  Parity with SCN itself stays "unpinned"
(SURVEY.md §8(c)); what is pinned here is the arithmetic under SCN's
documented conventions (last-axis-fastest filter offsets, size==stride
strided conv, biased-variance BN with unbiased running variance).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import scn_oracle as O
from oracle.encoders import OracleEncoder

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cloud(n=400, S=12, B=2, C=4, seed=0):
    rng = np.random.default_rng(seed)
    c = np.concatenate([rng.integers(0, S, (n, 3)), rng.integers(0, B, (n, 1))], 1)
    f = torch.from_numpy(rng.standard_normal((n, C)))
    return torch.from_numpy(c), f


def _dense(t, S, B):
    lvl = t.metadata.levels[t.size]
    c = lvl.coords
    d = torch.zeros(B, t.features.shape[1], S, S, S, dtype=t.features.dtype)
    d[c[:, 3], :, c[:, 0], c[:, 1], c[:, 2]] = t.features
    return d


def _at_sites(dense, t):
    c = t.metadata.levels[t.size].coords
    return dense[c[:, 3], :, c[:, 0], c[:, 1], c[:, 2]]


@pytest.mark.parametrize("cin,cout,f", [(4, 5, 3), (4, 2, 1), (3, 6, 5)])
def test_subm_equals_dense_conv(cin, cout, f):
    torch.manual_seed(cin + f)
    c, x = _cloud(C=cin)
    t = O.InputLayer(3, 12, mode=4)([c, x])
    conv = O.SubmanifoldConvolution(3, cin, cout, f, False).double()
    y = conv(t).features
    w = conv.weight[:, 0].reshape(f, f, f, cin, cout).permute(4, 3, 0, 1, 2)
    ref = _at_sites(F.conv3d(_dense(t, 12, 2), w, padding=f // 2), t)
    assert torch.allclose(y, ref, atol=1e-12)


@pytest.mark.parametrize("s", [2, 4])
def test_strided_conv_deconv_equal_dense(s):
    torch.manual_seed(s)
    c, x = _cloud(S=16)
    t = O.InputLayer(3, 16, mode=4)([c, x])
    conv = O.Convolution(3, 4, 6, s, s, False).double()
    z = conv(t)
    w = conv.weight[:, 0].reshape(s, s, s, 4, 6).permute(4, 3, 0, 1, 2)
    assert torch.allclose(z.features, _at_sites(F.conv3d(_dense(t, 16, 2), w, stride=s), z), atol=1e-12)
    de = O.Deconvolution(3, 6, 3, s, s, False).double()
    u = de(z)
    wt = de.weight[:, 0].reshape(s, s, s, 6, 3).permute(3, 4, 0, 1, 2)
    ref = _at_sites(F.conv_transpose3d(_dense(z, 16 // s, 2), wt, stride=s), u)
    assert torch.allclose(u.features, ref, atol=1e-12)
    # UnPooling = copy of the parent row; MaxPooling = dense max over the block
    up = O.UnPooling(3, s, s)(z)
    c_f = up.metadata.levels[16].coords
    par = z.metadata.levels[16 // s].lookup(np.concatenate([c_f[:, :3] // s, c_f[:, 3:]], 1))
    assert torch.equal(up.features, z.features[torch.from_numpy(par)])
    tp = O.InputLayer(3, 16, mode=4)([c, x.abs() + 0.1])
    mp = O.MaxPooling(3, s, s)(tp)
    assert torch.allclose(mp.features, _at_sites(F.max_pool3d(_dense(tp, 16, 2), s, s), mp))


def test_input_layer_known_answer():
    c = torch.tensor([[1, 2, 3, 0], [1, 2, 3, 0], [1, 2, 3, 1], [0, 0, 0, 0], [1, 2, 3, 0]])
    f = torch.tensor([[1.0], [2.0], [10.0], [5.0], [6.0]], dtype=torch.float64)
    t4 = O.InputLayer(3, 8, mode=4)([c, f])
    t3 = O.InputLayer(3, 8, mode=3)([c, f])
    # raster order: (b0,0,0,0), (b0,1,2,3), (b1,1,2,3)
    assert t4.features.flatten().tolist() == [5.0, 3.0, 10.0]
    assert t3.features.flatten().tolist() == [5.0, 9.0, 10.0]
    out = O.OutputLayer(3)(t4)
    assert out.flatten().tolist() == [3.0, 3.0, 10.0, 5.0, 3.0]


def test_subm_rule_counts_known_answer():
    # an L-shape of 3 voxels: (0,0,0) - (1,0,0) - (1,1,0)
    c = torch.tensor([[0, 0, 0, 0], [1, 0, 0, 0], [1, 1, 0, 0]])
    t = O.InputLayer(3, 4, mode=4)([c, torch.ones(3, 1, dtype=torch.float64)])
    rules = t.metadata.levels[4].subm_rules(3)
    counts = [len(a) for a, _ in rules]
    # centre + every pair within the 3x3x3 box both ways ((0,0,0)-(1,1,0) is a diagonal neighbour)
    assert counts[13] == 3 and sum(counts) == 3 + 3 * 2
    # offset index of (dx, dy, dz) = ((dx+1)*3 + dy+1)*3 + dz+1; (1,0,0) is a +x neighbour of (0,0,0)
    o = (2 * 3 + 1) * 3 + 1
    a, b = rules[o]
    assert list(zip(a.tolist(), b.tolist())) == [(1, 0)]


def test_batchnorm_matches_torch():
    torch.manual_seed(0)
    c, x = _cloud(C=6)
    t = O.InputLayer(3, 12, mode=4)([c, x * 2 + 1])
    bn = O.BatchNormLeakyReLU(6, leakiness=0.2).double()
    with torch.no_grad():
        bn.weight.copy_(torch.linspace(0.5, 1.5, 6))
        bn.bias.copy_(torch.linspace(-1, 1, 6))
    y = bn(t).features
    rm, rv = torch.zeros(6, dtype=torch.float64), torch.ones(6, dtype=torch.float64)
    ref = F.batch_norm(t.features, rm, rv, bn.weight, bn.bias, training=True, momentum=0.1, eps=1e-4)
    assert torch.allclose(y, F.leaky_relu(ref, 0.2), atol=1e-12)
    # SCN momentum 0.9 == torch momentum 0.1; both use the unbiased running variance
    assert torch.allclose(bn.running_mean.double(), rm, atol=1e-7)
    assert torch.allclose(bn.running_var.double(), rv, atol=1e-6)
    bn.eval()
    ye = bn(t).features
    refe = F.batch_norm(t.features, rm, rv, bn.weight, bn.bias, training=False, eps=1e-4)
    assert torch.allclose(ye, F.leaky_relu(refe, 0.2), atol=1e-6)


@pytest.mark.parametrize("tag", ["c1_fcnencoder", "c2_unet_m16", "c3_unet_m32_res"])
def test_oracle_reproduces_golden(tag):
    z = np.load(os.path.join(GOLD, f"oracle_{tag}.npz"))
    name, m, reps, res, seed = z["meta"].tolist()
    torch.manual_seed(int(seed))
    ref = OracleEncoder(name, m=int(m), block_reps=int(reps), residual_blocks=bool(int(res)))
    chk = float(sum(p.detach().double().sum() for p in ref.parameters()))
    assert abs(chk - float(z["param_checksum"])) < 1e-9 * max(1.0, abs(chk))
    ref = ref.double()
    x = dict(coords=torch.from_numpy(z["coords"].astype(np.int64)), feature=torch.from_numpy(z["feats"]).double(),
             batch_offsets=z["batch_offsets"].tolist())
    pp = ref(x)
    glob = ref(x, istrain=True)
    (glob * torch.linspace(-1, 1, glob.shape[1], dtype=torch.float64)).sum().backward()
    assert np.allclose(pp.detach().numpy()[z["rows"]], z["per_point"], atol=1e-10)
    assert np.allclose(glob.detach().numpy(), z["scene"], atol=1e-10)
    assert np.allclose(ref.encoder[1].weight.grad.numpy(), z["grad_first"], atol=1e-10)


@pytest.mark.parametrize("train", [True, False])
def test_lean_adjoints_equal_autograd(train):
    """The oracle's hand-written adjoints (LEAN: submanifold convolution and BatchNorm-(leaky)ReLU saving only their
    inputs, oracle/scn_oracle.py) give the forward and every parameter / input gradient of autograd over the
    plain op composition, on a residual UNet with leaky ReLUs (fp64, 1e-12 relative)."""
    from wsss3d.synthetic import make_batch
    b = make_batch(2, 8, seed=5, spacing=0.04)
    coords = torch.from_numpy(b["coords"])
    outs = {}
    for lean in (False, True):
        O.LEAN = lean
        try:
            torch.manual_seed(3)
            ref = OracleEncoder("SparseConvUNet", m=8, block_reps=2, residual_blocks=True).double()
            for mod in ref.modules():  # leaky ReLUs and non-trivial affines exercise every term
                if isinstance(mod, O.BatchNormalization):
                    mod.leak = 0.1
                    with torch.no_grad():
                        mod.weight.uniform_(0.5, 1.5)
                        mod.bias.uniform_(-0.2, 0.2)
            ref.train(train)
            feats = torch.from_numpy(b["feats"]).double().requires_grad_(True)
            x = dict(coords=coords, feature=feats, batch_offsets=b["batch_offsets"])
            out = ref(x, istrain=True)
            w = torch.linspace(-1, 1, out.numel(), dtype=torch.float64).view_as(out)
            (out * w).sum().backward()
            outs[lean] = (out.detach(), feats.grad, {k: p.grad for k, p in ref.named_parameters()})
        finally:
            O.LEAN = True
    (o0, f0, g0), (o1, f1, g1) = outs[False], outs[True]
    assert torch.allclose(o1, o0, rtol=0, atol=1e-12 * o0.abs().max().item())
    assert torch.allclose(f1, f0, rtol=0, atol=1e-12 * f0.abs().max().item())
    for k in g0:
        assert torch.allclose(g1[k], g0[k], rtol=0, atol=1e-12 * max(g0[k].abs().max().item(), 1e-30)), k
