"""Op-level parity of the HIP path against the CPU oracle (fp64).

Tolerances: features/gradients are fp32 on the device and fp64 in the oracle;
each check is max|gpu - oracle| <= tol * max(1, max|oracle|) with tol = 1e-5
for single ops (one fp32 contraction) unless stated.  Integer metadata
(voxel sets, per-offset rule counts, child maps) must match exactly.
"""
import numpy as np
import pytest
import torch

import sparseconvnet as scn
from oracle import scn_oracle as O
from wsss3d.synthetic import make_batch, random_cloud

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def close(a, b, tol=1e-5, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item() if a.numel() else 0.0
    lim = tol * max(1.0, b.abs().max().item() if b.numel() else 0.0)
    assert err <= lim, f"{what}: max err {err:.3e} > {lim:.3e}"


def _inputs(n=3000, extent=24, n_batch=2, n_feat=3, seed=0):
    coords, feats = random_cloud(n, extent, n_batch=n_batch, seed=seed, n_feat=n_feat, dense_frac=0.3)
    return torch.from_numpy(coords), torch.from_numpy(feats)


def _pair(coords, feats, size=32, mode=4, same_input=True):
    """InputLayer on both sides; with same_input the oracle continues from the
    device's voxel features (so each op test isolates that op's error from the
    fp32 averaging of the input layer)."""
    g = scn.InputLayer(3, size, mode=mode)([coords.to(DEV), feats.to(DEV)])
    o = O.InputLayer(3, size, mode=mode)([coords, feats.double()])
    if same_input:
        o.features = _to_oracle_order(g, o).detach().double().cpu()
    return g, o


def _to_oracle_order(g_tensor, o_tensor):
    """Rows of the GPU tensor permuted into the oracle's (raster) row order."""
    loc = g_tensor.get_spatial_locations().cpu().numpy()
    lvl = o_tensor.metadata.levels[o_tensor.size]
    idx = lvl.lookup(loc)
    assert (idx >= 0).all() and len(np.unique(idx)) == lvl.n == len(loc)
    perm = np.empty(lvl.n, np.int64)
    perm[idx] = np.arange(len(loc))
    return g_tensor.features[torch.from_numpy(perm).to(g_tensor.features.device)]


@pytest.mark.parametrize("mode", [3, 4])
def test_input_output_layer(mode):
    coords, feats = _inputs()
    g, o = _pair(coords, feats, mode=mode, same_input=False)
    assert g.features.shape[0] == o.features.shape[0]
    close(_to_oracle_order(g, o), o.features, 1e-6, "input features")
    out_g = scn.OutputLayer(3)(g)
    out_o = O.OutputLayer(3)(o)
    close(out_g, out_o, 1e-6, "output layer")


def test_input_layer_backward():
    coords, feats = _inputs()
    fg = feats.to(DEV).requires_grad_(True)
    fo = feats.double().requires_grad_(True)
    g = scn.InputLayer(3, 32, mode=4)([coords.to(DEV), fg])
    o = O.InputLayer(3, 32, mode=4)([coords, fo])
    w = torch.randn(g.features.shape[1], 5, dtype=torch.float64)
    (scn.OutputLayer(3)(g) @ w.float().to(DEV)).square().sum().backward()
    (O.OutputLayer(3)(o) @ w).square().sum().backward()
    close(fg.grad, fo.grad, 1e-5, "input grad")


def test_levels_match_oracle():
    coords, feats = _inputs(5000, 60, n_batch=3)
    g, o = _pair(coords, feats, size=64)
    meta_g, meta_o = g.metadata, o.metadata
    size = 64
    while size >= 2:
        lg = meta_g.locations(size).cpu().numpy()
        lo = meta_o.levels[size].coords
        key = lambda c: np.lexsort((c[:, 2], c[:, 1], c[:, 0], c[:, 3]))  # noqa: E731
        assert np.array_equal(lg[key(lg)], lo[key(lo)]), f"level {size}"
        rg = meta_g.level(size).subm_rules(3)
        ro = meta_o.levels[size].subm_rules(3)
        assert rg.pairs.counts == [len(a) for a, _ in ro], f"rule counts at {size}"
        assert rg.pairs.counts == rg.pairs.counts[::-1]  # symmetric neighbourhoods
        meta_g.downsample(size, 2)
        meta_o.downsample(size, 2)
        size //= 2


@pytest.mark.parametrize("cin,cout", [(3, 16), (3, 32), (1, 64), (4, 32), (16, 16), (32, 32), (64, 32), (48, 96), (32, 224)])
def test_subm_conv(cin, cout):
    torch.manual_seed(cin * 1000 + cout)
    coords, feats = _inputs(4000, 28, n_feat=cin)
    g, o = _pair(coords, feats)
    conv_g = scn.SubmanifoldConvolution(3, cin, cout, 3, False).to(DEV)
    conv_o = O.SubmanifoldConvolution(3, cin, cout, 3, False).double()
    conv_o.weight.data.copy_(conv_g.weight.data.double().cpu())
    xg = g.features.detach().requires_grad_(True)
    xo = o.features.detach().requires_grad_(True)
    g.features, o.features = xg, xo
    yg, yo = conv_g(g), conv_o(o)
    close(_to_oracle_order(yg, yo), yo.features, 1e-5, "subm fwd")
    w = torch.randn(cout, dtype=torch.float64)
    (yg.features * w.float().to(DEV)).square().sum().backward()
    (yo.features * w).square().sum().backward()
    close(_to_oracle_order(type(g)(xg.grad, g.metadata, g.spatial_size), o), xo.grad, 1e-5, "subm dx")
    close(conv_g.weight.grad, conv_o.weight.grad, 1e-5, "subm dW")


@pytest.mark.parametrize("stride,cin,cout", [(2, 16, 32), (2, 32, 48), (4, 32, 64), (2, 32, 64), (2, 64, 96)])
def test_strided_conv_deconv_unpool(stride, cin, cout):
    """Strided convolution, deconvolution, unpooling and max pooling against the oracle, forward and backward.
    (2, 32, 64) and (2, 64, 96) also run with the chunk weight gradient over the child map for both the
    convolution and the deconvolution (round 6, opt-in; channels in multiples of 32)."""
    torch.manual_seed(stride + cin)
    coords, feats = _inputs(4000, 40, n_feat=cin)
    g, o = _pair(coords, feats, size=64)
    xg = g.features.detach().requires_grad_(True)
    xo = o.features.detach().requires_grad_(True)
    g.features, o.features = xg, xo
    cg = scn.Convolution(3, cin, cout, stride, stride, False).to(DEV)
    co = O.Convolution(3, cin, cout, stride, stride, False).double()
    co.weight.data.copy_(cg.weight.data.double().cpu())
    dg = scn.Deconvolution(3, cout, cin, stride, stride, False).to(DEV)
    do = O.Deconvolution(3, cout, cin, stride, stride, False).double()
    do.weight.data.copy_(dg.weight.data.double().cpu())
    zg, zo = cg(g), co(o)
    assert int(zg.spatial_size[0]) == 64 // stride
    close(_to_oracle_order(zg, zo), zo.features, 1e-5, "conv fwd")
    ug, uo = dg(zg), do(zo)
    close(_to_oracle_order(ug, uo), uo.features, 1e-5, "deconv fwd")
    pg, po = scn.UnPooling(3, stride, stride)(zg), O.UnPooling(3, stride, stride)(zo)
    close(_to_oracle_order(pg, po), po.features, 1e-6, "unpool fwd")
    mg, mo = scn.MaxPooling(3, stride, stride)(g), O.MaxPooling(3, stride, stride)(o)
    close(_to_oracle_order(mg, mo), mo.features, 1e-6, "maxpool fwd")
    w1 = torch.randn(cin, dtype=torch.float64)
    lg = (ug.features * w1.float().to(DEV)).square().sum() + pg.features.sum() + mg.features.square().sum()
    lo = (uo.features * w1).square().sum() + po.features.sum() + mo.features.square().sum()
    lg.backward()
    lo.backward()
    close(_to_oracle_order(type(g)(xg.grad, g.metadata, g.spatial_size), o), xo.grad, 1e-5, "dx")
    close(cg.weight.grad, co.weight.grad, 1e-5, "conv dW")
    close(dg.weight.grad, do.weight.grad, 1e-5, "deconv dW")
    if stride == 2 and cin % 32 == 0 and cout % 32 == 0:  # the opt-in chunk form over the child map
        from sparseconvnet import ops
        ops.STRIDED_WGRAD_CHUNK = True
        try:
            for m in (cg, dg):
                m.weight.grad = None
            xg.grad = None
            ug2 = dg(cg(g))
            pg2 = scn.UnPooling(3, stride, stride)(cg(g))
            mg2 = scn.MaxPooling(3, stride, stride)(g)
            ((ug2.features * w1.float().to(DEV)).square().sum() + pg2.features.sum() +
             mg2.features.square().sum()).backward()
        finally:
            ops.STRIDED_WGRAD_CHUNK = False
        close(cg.weight.grad, co.weight.grad, 1e-5, "conv dW (chunk form)")
        close(dg.weight.grad, do.weight.grad, 1e-5, "deconv dW (chunk form)")


@pytest.mark.parametrize("cin,cout", [(32, 64), (64, 32)])
def test_strided_wgrad_chunk_dense_children(cin, cout):
    """The chunk weight gradient over the child map where every coarse site has all 8 children (a solid block):
    a 128-coarse-row tile names up to 1024 distinct fine rows, past the 448 the kernel stages, so most rules go
    through the far-rule path (msp_wgrad_far_list + msp_conv_wgrad_far).  Convolution and deconvolution weight
    gradients against fp64 (1e-5 of the max), and the pair-list form agrees."""
    from sparseconvnet import ops
    torch.manual_seed(cin + cout)
    g0 = np.stack(np.meshgrid(*[np.arange(20)] * 3, indexing="ij"), -1).reshape(-1, 3)
    coords = torch.from_numpy(np.concatenate([g0, np.zeros((len(g0), 1), np.int64)], 1))
    feats = torch.randn(len(g0), cin)
    g, o = _pair(coords, feats, size=32)
    outs = []
    for chunk in (True, False):
        ops.STRIDED_WGRAD_CHUNK = chunk
        try:
            torch.manual_seed(5)
            cg = scn.Convolution(3, cin, cout, 2, 2, False).to(DEV)
            dg = scn.Deconvolution(3, cout, cin, 2, 2, False).to(DEV)
            xg = g.features.detach().requires_grad_(True)
            t = type(g)(xg, g.metadata, g.spatial_size)
            u = dg(cg(t))
            (u.features * torch.linspace(-1, 1, u.features.numel(), device=DEV).view_as(u.features)).sum().backward()
            outs.append((cg.weight.grad.clone(), dg.weight.grad.clone()))
            if chunk:
                rules = g.metadata.downsample(32, 2)[1]
                idx = rules.wgrad_index(wait=True)
                assert idx is not None and idx["n_far"] > 0, "the dense block must exercise the far-rule path"
        finally:
            ops.STRIDED_WGRAD_CHUNK = False
    co = O.Convolution(3, cin, cout, 2, 2, False).double()
    do = O.Deconvolution(3, cout, cin, 2, 2, False).double()
    torch.manual_seed(5)
    co.weight.data.copy_(scn.Convolution(3, cin, cout, 2, 2, False).weight.data.double())
    do.weight.data.copy_(scn.Deconvolution(3, cout, cin, 2, 2, False).weight.data.double())
    xo = o.features.detach().requires_grad_(True)
    uo = do(co(type(o)(xo, o.metadata, o.size)))
    # the device's loss weights (a linspace over its output rows) in the oracle's row order
    (uo.features * _device_weights_in_oracle_order(u, uo)).sum().backward()
    close(outs[0][0], co.weight.grad, 1e-5, "conv dW (chunk form)")
    close(outs[0][1], do.weight.grad, 1e-5, "deconv dW (chunk form)")
    close(outs[0][0], outs[1][0], 1e-5, "conv dW chunk vs pairs")
    close(outs[0][1], outs[1][1], 1e-5, "deconv dW chunk vs pairs")


def _device_weights_in_oracle_order(u, uo):
    """The per-element loss weights the device run used (linspace over its rows), permuted into the oracle's
    row order."""
    w = torch.linspace(-1, 1, u.features.numel(), device=DEV).view_as(u.features)
    return _to_oracle_order(type(u)(w, u.metadata, u.spatial_size), uo).double().cpu()


@pytest.mark.parametrize("cin,cout", [(64, 32), (96, 64), (48, 16), (160, 32)])
def test_conv_pairs_runs_cross_offsets(cin, cout):
    """msp_conv_pairs at a size where a wave takes a run of chunks with the weights in registers (c_in <= 64),
    runs crossing from one offset into the next and over an empty offset, against fp64: every output row has one
    contribution, W[o]^T x[pin], as the deconvolution forward and the strided backward-data have.  c_in = 96 and
    160 take the one-chunk form.  The library's f32 MFMA products are exact, so 1e-5 is the fp32 accumulation; the
    split-bf16 form (msp_conv_pairs_x6, the production path since round 6) is held to the same bar."""
    from sparseconvnet import _lib
    g = torch.Generator().manual_seed(cin + cout)
    K, n_out, n_in = 8, 300_000, 50_000
    counts = torch.multinomial(torch.ones(K), n_out, replacement=True, generator=g).bincount(minlength=K)
    counts[3] = 0   # an empty offset
    counts[0] += n_out - int(counts.sum())
    starts = torch.zeros(K + 1, dtype=torch.int64)
    starts[1:] = counts.cumsum(0)
    pout = torch.randperm(n_out, generator=g).int()
    pin = torch.randint(0, n_in, (n_out,), generator=g).int()
    for o in range(K):  # sorted by source row within an offset, as the pair lists are
        a, b = int(starts[o]), int(starts[o + 1])
        pin[a:b] = pin[a:b].sort().values
    chunk_start = torch.zeros(K + 1, dtype=torch.int64)
    chunk_start[1:] = ((counts + 15) // 16).cumsum(0)
    n_chunks = int(chunk_start[-1])
    x = torch.randn(n_in, cin, generator=g)
    wt = torch.randn(K, cout, cin, generator=g)   # [K][c_out][c_in]
    dx, dwt, dpin, dpout = x.to(DEV), wt.to(DEV), pin.to(DEV), pout.to(DEV)
    dst, dcs = starts.to(DEV), chunk_start.to(DEV)
    out = torch.full((n_out, cout), float("nan"), device=DEV)
    _lib.call("msp_conv_pairs", dx.data_ptr(), cin, dwt.data_ptr(), K, cout, dpin.data_ptr(), dpout.data_ptr(),
              dst.data_ptr(), dcs.data_ptr(), n_chunks, out.data_ptr(), _lib.stream())
    torch.cuda.synchronize()
    ref = torch.empty(n_out, cout, dtype=torch.float64)
    for o in range(K):
        a, b = int(starts[o]), int(starts[o + 1])
        ref[pout[a:b].long()] = x[pin[a:b].long()].double() @ wt[o].double().t()
    close(out, ref, 1e-5, f"conv_pairs {cin}->{cout}")
    # the split-bf16 form (msp_conv_pairs_x6): three-piece products, one zeroed accumulator per 32-deep slice
    wsb = int(_lib.query("msp_conv_pairs_x6_workspace_size", K, cin, cout))
    ws = torch.empty(wsb // 4 + 4, dtype=torch.float32, device=DEV)
    out6 = torch.full((n_out, cout), float("nan"), device=DEV)
    _lib.call("msp_conv_pairs_x6", dx.data_ptr(), cin, dwt.data_ptr(), K, cout, dpin.data_ptr(), dpout.data_ptr(),
              dst.data_ptr(), dcs.data_ptr(), n_chunks, out6.data_ptr(), ws.data_ptr(), wsb, _lib.stream())
    torch.cuda.synchronize()
    close(out6, ref, 1e-5, f"conv_pairs_x6 {cin}->{cout}")


@pytest.mark.parametrize("cin,cout,K,counts", [
    (16, 16, 1, [1]),                       # one pair, one offset
    (32, 48, 8, [0, 17, 0, 0, 33, 1, 0, 16]),  # empty offsets first and between, partial chunks (NT = 1 of 3 tiles)
    (144, 48, 8, [5, 0, 40, 3, 0, 0, 70, 2]),  # c_in > 128: one chunk per wave; 144 = 4.5 slices (zero-padded k)
    (128, 80, 27, None),                      # c_in = 128 (four slices in registers), c_out 80 (NT = 1, 5 column tiles)
])
def test_conv_pairs_x6_edges(cin, cout, K, counts):
    """msp_conv_pairs_x6 at the edges of its forms against fp64 (1e-5 of the max): a single pair, empty offsets at
    the start and between (a wave's run crosses them), partial last chunks, c_in past the register-run form's 128,
    and column tiles of 16 (odd c_out / 16).  Output rows no pair names stay untouched (NaN sentinel)."""
    from sparseconvnet import _lib
    g = torch.Generator().manual_seed(cin * 7 + cout + K)
    if counts is None:
        counts = torch.randint(0, 400, (K,), generator=g).tolist()
    counts = torch.tensor(counts, dtype=torch.int64)
    n_pairs = int(counts.sum())
    n_out, n_in = n_pairs + 37, max(n_pairs // 2, 1) + 5
    starts = torch.zeros(K + 1, dtype=torch.int64)
    starts[1:] = counts.cumsum(0)
    pout = torch.randperm(n_out, generator=g)[:n_pairs].int()
    pin = torch.randint(0, n_in, (n_pairs,), generator=g).int()
    chunk_start = torch.zeros(K + 1, dtype=torch.int64)
    chunk_start[1:] = ((counts + 15) // 16).cumsum(0)
    n_chunks = int(chunk_start[-1])
    x = torch.randn(n_in, cin, generator=g)
    wt = torch.randn(K, cout, cin, generator=g)
    wsb = int(_lib.query("msp_conv_pairs_x6_workspace_size", K, cin, cout))
    ws = torch.empty(wsb // 4 + 4, dtype=torch.float32, device=DEV)
    out = torch.full((n_out, cout), float("nan"), device=DEV)
    dx, dwt, dpin, dpout = x.to(DEV), wt.to(DEV), pin.to(DEV), pout.to(DEV)
    dst, dcs = starts.to(DEV), chunk_start.to(DEV)
    _lib.call("msp_conv_pairs_x6", dx.data_ptr(), cin, dwt.data_ptr(), K, cout, dpin.data_ptr(), dpout.data_ptr(),
              dst.data_ptr(), dcs.data_ptr(), n_chunks, out.data_ptr(), ws.data_ptr(), wsb, _lib.stream())
    torch.cuda.synchronize()
    ref = torch.full((n_out, cout), float("nan"), dtype=torch.float64)
    for o in range(K):
        a, b = int(starts[o]), int(starts[o + 1])
        ref[pout[a:b].long()] = x[pin[a:b].long()].double() @ wt[o].double().t()
    named = torch.zeros(n_out, dtype=torch.bool)
    named[pout.long()] = True
    o_cpu = out.double().cpu()
    assert torch.isnan(o_cpu[~named]).all(), "rows no pair names were written"
    close(o_cpu[named], ref[named], 1e-5, f"conv_pairs_x6 edges {cin}->{cout} K={K}")


@pytest.mark.parametrize("C,leak,train,mu,sd", [(32, 0.0, True, 1.5, 3.0), (48, 0.333, True, 1.5, 3.0),
                                                (896, 0.0, True, 1.5, 3.0), (16, 0.0, False, 1.5, 3.0),
                                                (32, 0.0, True, 10.0, 0.01)])
def test_batchnorm(C, leak, train, mu, sd):
    """Last case: low-variance channels far from zero (mean/std = 1e3), where
    folding the mean into the shift loses the ReLU decision (kept as a
    regression test for that bug)."""
    torch.manual_seed(C)
    coords, feats = _inputs(3000, 24, n_feat=C)
    feats = feats * sd + mu
    g, o = _pair(coords, feats)
    bg = scn.BatchNormLeakyReLU(C, leakiness=leak).to(DEV)
    bo = O.BatchNormLeakyReLU(C, leakiness=leak).double()
    with torch.no_grad():
        for b in (bg, bo):
            b.weight.copy_(torch.linspace(0.5, 1.5, C))
            b.bias.copy_(torch.linspace(-0.2, 0.3, C))
            b.running_mean.copy_(torch.linspace(-1, 1, C))
            b.running_var.copy_(torch.linspace(0.5, 2, C))
    bg.train(train)
    bo.train(train)
    xg = g.features.detach().requires_grad_(True)
    xo = o.features.detach().requires_grad_(True)
    g.features, o.features = xg, xo
    yg, yo = bg(g), bo(o)
    close(_to_oracle_order(yg, yo), yo.features, 2e-5, "bn fwd")
    w = torch.randn(C, dtype=torch.float64)
    (yg.features * w.float().to(DEV)).square().sum().backward()
    (yo.features * w).square().sum().backward()
    close(_to_oracle_order(type(g)(xg.grad, g.metadata, g.spatial_size), o), xo.grad, 2e-5, "bn dx")
    close(bg.weight.grad, bo.weight.grad, 2e-5, "bn dweight")
    close(bg.bias.grad, bo.bias.grad, 2e-5, "bn dbias")
    close(bg.running_mean, bo.running_mean, 1e-6, "running mean")
    close(bg.running_var, bo.running_var, 1e-6, "running var")


def test_nin_join_add():
    coords, feats = _inputs(2000, 20, n_feat=32)
    g, _ = _pair(coords, feats)
    nin = scn.NetworkInNetwork(32, 16, False).to(DEV)
    y = nin(g)
    torch.testing.assert_close(y.features, g.features @ nin.weight)
    j = scn.JoinTable()([g, y])
    assert j.features.shape[1] == 48
    a = scn.AddTable()([y, y])
    torch.testing.assert_close(a.features, 2 * y.features)


@pytest.mark.parametrize("ca,cb", [(32, 32), (64, 128), (16, 8), (6, 10)])
def test_join_table(ca, cb):
    """JoinTable on msp_join_cols: bit-equal to torch.cat in branch order, its backward bit-equal to the gradient's
    column slices (msp_split_cols), and the batch-statistic partials it leaves in training mode give the following
    BatchNormalization bit-identical outputs, gradients and running statistics to the BN's own statistics pass
    (FUSE_RESIDUAL off)."""
    from sparseconvnet import modules as M
    coords, feats = _inputs(5000, 24, n_feat=ca)
    torch.manual_seed(ca + cb)
    outs = []
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    b0 = torch.randn(t.features.size(0), cb, device=DEV)
    g = torch.randn(t.features.size(0), ca + cb, device=DEV)
    for fuse in (True, False):
        M.FUSE_RESIDUAL = fuse
        try:
            a = t.features.detach().clone().requires_grad_(True)
            b = b0.clone().requires_grad_(True)
            ta = scn.SparseConvNetTensor(a, t.metadata, t.spatial_size)
            tb = scn.SparseConvNetTensor(b, t.metadata, t.spatial_size)
            j = scn.JoinTable().train()([ta, tb])
            assert torch.equal(j.features, torch.cat([a, b], 1))
            assert (getattr(j, "_bn_partial", None) is not None) == fuse
            bn = scn.BatchNormReLU(ca + cb).to(DEV)
            y = bn(j).features
            y.backward(g)
            outs.append((y.detach(), a.grad, b.grad, bn.weight.grad, bn.running_mean.clone(), bn.running_var.clone()))
        finally:
            M.FUSE_RESIDUAL = True
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    gj = torch.randn(a.size(0), ca + cb, device=DEV)
    ga, gb = torch.autograd.grad(scn.JoinTable()([ta, tb]).features, (a, b), gj)
    assert torch.equal(ga, gj[:, :ca]) and torch.equal(gb, gj[:, ca:])


@pytest.mark.parametrize("n,cin,cout", [(5000, 64, 32), (3001, 40, 24), (70000, 96, 48)])
def test_nin_grads(n, cin, cout):
    """NetworkInNetwork backward: dx on msp_nin_gemm, dW on msp_conv_wgrad with
    identity pairs (any channel counts: padded to 16), against fp64 torch."""
    torch.manual_seed(n)
    coords, feats = _inputs(n, 30, n_feat=cin)
    g, _ = _pair(coords, feats)
    nin = scn.NetworkInNetwork(cin, cout, False).to(DEV)
    x = g.features.detach().requires_grad_(True)
    g.features = x
    y = nin(g).features
    w = torch.randn(cout, device=DEV)
    (y * w).square().sum().backward()
    xd, wd = x.detach().double(), nin.weight.detach().double()
    yd = xd @ wd
    gy = 2 * yd * w.double().square()
    close(x.grad, gy @ wd.t(), 1e-5, "nin dx")
    close(nin.weight.grad, xd.t() @ gy, 1e-5, "nin dW")


def test_empty_and_single_point():
    c = torch.tensor([[5, 6, 7, 0]])
    f = torch.randn(1, 3)
    net = scn.Sequential(scn.InputLayer(3, 16, mode=4), scn.SubmanifoldConvolution(3, 3, 16, 3, False),
                         scn.BatchNormReLU(16), scn.OutputLayer(3)).to(DEV)
    out = net([c.to(DEV), f.to(DEV)])
    assert out.shape == (1, 16) and torch.isfinite(out).all()
    with pytest.raises(ValueError):
        scn.InputLayer(3, 16, mode=4)([torch.tensor([[16, 0, 0, 0]]).to(DEV), f.to(DEV)])


def test_cpu_tensor_fails_loudly():
    coords, feats = _inputs(100, 8)
    with pytest.raises(RuntimeError):
        scn.InputLayer(3, 16, mode=4)([coords, feats])


def test_full_size_determinism_and_invariants():
    """C3-sized batch: metadata invariants and bitwise-repeatable forward."""
    b = make_batch(8, 50, seed=1)
    coords = torch.from_numpy(b["coords"]).to(DEV)
    feats = torch.from_numpy(b["feats"]).to(DEV)
    conv = scn.SubmanifoldConvolution(3, 3, 32, 3, False).to(DEV)
    outs = []
    for _ in range(2):
        t = scn.InputLayer(3, 4096, mode=4)([coords, feats])
        outs.append(conv(t).features)
    assert torch.equal(outs[0], outs[1])
    lvl = t.metadata.level(4096)
    r = lvl.subm_rules(3)
    assert r.pairs.counts[13] == lvl.n  # centre offset always present
    assert r.pairs.counts == r.pairs.counts[::-1]
    coarse, d = t.metadata.downsample(4096, 2)
    assert sum(d.pairs.counts) == lvl.n  # every fine site has exactly one parent
    cs = d.child_start.cpu()
    assert cs[0] == 0 and cs[-1] == lvl.n and bool((cs[1:] > cs[:-1]).all())


@pytest.mark.parametrize("n,cin", [(3000, 64), (12000, 64), (12000, 32)])
def test_residual_block_grads(n, cin):
    """ConcatTable(NIN | BN-SubM-BN-SubM) + AddTable: the UNet decoder block
    whose input gradient sums two branches (models/SparseConvNet.py:112-120)."""
    torch.manual_seed(n + cin)
    coords, feats = _inputs(n, 40, n_feat=cin)
    g, o = _pair(coords, feats, size=64)

    def block(lib, a, b):
        sc = lib.NetworkInNetwork(a, b, False) if a != b else lib.Identity()
        return lib.Sequential().add(lib.ConcatTable().add(sc).add(
            lib.Sequential().add(lib.BatchNormReLU(a)).add(lib.SubmanifoldConvolution(3, a, b, 3, False))
            .add(lib.BatchNormReLU(b)).add(lib.SubmanifoldConvolution(3, b, b, 3, False)))).add(lib.AddTable())

    bg = block(scn, cin, 32).to(DEV)
    bo = block(O, cin, 32).double()
    bo.load_state_dict({k: v.double().cpu() for k, v in bg.state_dict().items()})
    xg = g.features.detach().requires_grad_(True)
    xo = o.features.detach().requires_grad_(True)
    g.features, o.features = xg, xo
    yg, yo = bg(g), bo(o)
    close(_to_oracle_order(yg, yo), yo.features, 1e-5, "block fwd")
    w = torch.randn(32, dtype=torch.float64)
    (yg.features * w.float().to(DEV)).square().sum().backward()
    (yo.features * w).square().sum().backward()
    close(_to_oracle_order(type(g)(xg.grad, g.metadata, g.spatial_size), o), xo.grad, 1e-4, "block dx")
    pg = dict(bg.named_parameters())
    for k, p in bo.named_parameters():
        close(pg[k].grad, p.grad, 1e-4, "grad " + k)


def _subm_ref(x, wt, nbr, flip, dtype):
    """sum over offsets of x[nbr(., o)] W'[o]^T evaluated by torch in `dtype` (fp64: the reference; fp32: a plain
    fp32 evaluation whose error the split-bf16 kernels are held to); wt [K][c_out][c_in], flip mirrors offsets."""
    V, K = nbr.size(1), nbr.size(0)
    xd = torch.cat([x.to(dtype), torch.zeros(1, x.size(1), dtype=dtype, device=x.device)])
    wd = wt.to(dtype).flip(0) if flip else wt.to(dtype)
    nb = nbr.long()
    ref = torch.zeros(V, wt.size(1), dtype=dtype, device=x.device)
    for o in range(K):
        ref += xd[torch.where(nb[o] >= 0, nb[o], x.size(0))] @ wd[o].t()
    return ref


@pytest.mark.parametrize("cin,cout,flip", [(64, 64, 0), (96, 96, 1), (48, 96, 0), (256, 128, 0), (224, 32, 1),
                                           (32, 32, 0), (64, 32, 1), (48, 16, 0)])
def test_conv_tile_split_bf16_accuracy(cin, cout, flip):
    """msp_conv_tile on 128-row tiles runs the contraction as six bf16 MFMA
    products of exact three-piece splits (msp_conv_x6.hip).  Its error against
    an fp64 evaluation must be fp32-class: at most 3x that of a plain fp32
    evaluation (torch gather + fp32 GEMM) of the same sum, and below
    1e-6 of the output scale.  c_out <= 32 with c_in <= 64 takes the per-wave
    form (conv_x6r_kernel: weights per offset run), the rest the tile-local form,
    whose MFMAs accumulate the six piece products straight into the running sums
    (one rounding per product instead of per step: 1.5-3x the fp32 evaluation's
    error, measured 4.2e-7 / 7.0e-7 at 64->64 / 256->128)."""
    from sparseconvnet import ops
    torch.manual_seed(cin + cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    lvl = t.metadata.level(64)
    rules = lvl.subm_rules(3)
    V = lvl.n
    x = torch.randn(V, cin, device=DEV)
    wt = torch.randn(27, cout, cin, device=DEV) / (27 * cin) ** 0.5
    y = ops.conv_tile(x, wt, 27, flip, cout, rules, V)
    ref = _subm_ref(x, wt, rules.nbr, flip, torch.float64)
    y32 = _subm_ref(x, wt, rules.nbr, flip, torch.float32)
    scale = ref.abs().max().item()
    e_x6 = (y.double() - ref).abs().max().item() / scale
    e_f32 = (y32.double() - ref).abs().max().item() / scale
    print(f"conv_tile {cin}->{cout} flip {flip}: max err {e_x6:.2e} (fp32 evaluation {e_f32:.2e})")
    assert e_x6 <= max(3.0 * e_f32, 1e-7) and e_x6 < 1e-6, (e_x6, e_f32)


@pytest.mark.parametrize("cin,cout,flip", [(64, 64, 0), (64, 64, 1), (32, 64, 1), (96, 96, 0), (192, 96, 1),
                                           (96, 192, 0), (48, 64, 0), (64, 128, 1), (32, 32, 0), (16, 80, 1)])
def test_conv_nbr_accuracy(cin, cout, flip):
    """msp_conv_nbr (dense row groups over the neighbour map, register
    accumulators) against an fp64 evaluation of the same convolution: at most
    2x a plain fp32 evaluation's error and below 1e-6 of the output scale
    (this form sums each step's six piece products in a zeroed accumulator;
    the tile-local form, which chains them into the running sums, has the 3x
    bar of test_conv_tile_split_bf16_accuracy), and agreement
    with msp_conv_tile; the mask-sorted row order
    (msp_dense_order) gives bitwise the same rows.  Includes c_in not a
    multiple of 32 (zero k-padding) and a last group of rows past the level."""
    from sparseconvnet import _lib, ops
    from sparseconvnet._lib import ptr
    torch.manual_seed(cin * 7 + cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    lvl = t.metadata.level(64)
    rules = lvl.subm_rules(3)
    V = lvl.n
    assert V % 16 != 0 or V % 128 != 0  # a partial row group or block
    x = torch.randn(V, cin, device=DEV)
    wt = torch.randn(27, cout, cin, device=DEV) / (27 * cin) ** 0.5
    perm, nbr_p = rules.dense_order()
    assert sorted(perm.tolist()) == list(range(V))
    assert torch.equal(nbr_p, rules.nbr[:, perm.long()])
    y = ops.conv_nbr(x, wt, 27, flip, cout, rules.nbr, V)
    yp = ops.conv_nbr(x, wt, 27, flip, cout, nbr_p, V, perm=perm)
    tl = rules.tiles_for(128)
    yt = torch.empty(V, cout, device=DEV)
    wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(V), 27, cin, cout, 128))
    ws = torch.empty(max(wsb // 4, 1), device=DEV)
    _lib.call("msp_conv_tile", ptr(x), cin, ptr(wt), 27, flip, cout, 128, ptr(tl["tile_start"]),
              ptr(tl["chunk_off"]), ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(yt), ptr(ws), wsb,
              _lib.stream(x.device))
    ref = _subm_ref(x, wt, rules.nbr, flip, torch.float64)
    y32 = _subm_ref(x, wt, rules.nbr, flip, torch.float32)
    scale = ref.abs().max().item()
    e_g = (y.double() - ref).abs().max().item() / scale
    e_f32 = (y32.double() - ref).abs().max().item() / scale
    e_t = (yt.double() - ref).abs().max().item() / scale
    e_p = (yp.double() - ref).abs().max().item() / scale
    assert e_g <= max(2.0 * e_f32, 1e-7) and e_g < 1e-6, (e_g, e_f32, e_t)
    assert e_p <= max(2.0 * e_f32, 1e-7) and e_p < 1e-6, (e_p, e_f32, e_t)
    assert ((y - yt).abs().max().item() / scale) < 2e-6
    # same row groups' sums per row whatever the order: only the grouping of
    # zero rows differs, and zero products are exact
    assert torch.equal(y, yp)


def test_subm_conv_large_level_32_to_64():
    """A level above 10^5 rows with 32 -> 64 channels (level 0's decoder shape, below the tile-local form's 64 input
    channels) runs the module forward and the backward-data 64 -> 32 through the tile rulebook (the dense
    row-group form is off since round 5: msp_conv_nbr_preferred is 0), and msp_conv_nbr called directly on the
    map's dense row order gives the same output: output, input gradient and weight gradient match an fp64
    evaluation from the neighbour map (1e-5 of scale)."""
    from sparseconvnet import _lib, ops
    b = make_batch(1, 50, seed=5)
    coords = torch.from_numpy(b["coords"]).to(DEV)
    feats = torch.from_numpy(b["feats"]).to(DEV)
    t = scn.InputLayer(3, 4096, mode=4)([coords, feats])
    V = t.features.size(0)
    assert V >= 100000 and not int(_lib.query("msp_conv_nbr_preferred", _lib.I64(V), 32, 64))
    assert not int(_lib.query("msp_conv_local_preferred", _lib.I64(V), 32, 64))
    torch.manual_seed(3)
    x = torch.randn(V, 32, device=DEV, requires_grad=True)
    t.features = x

    class Kinds:
        def __init__(self):
            self.kinds = set()

        def run(self, kind, flops, fn, nbytes=0):
            self.kinds.add(kind.split("[")[0])
            return fn()
    rec = Kinds()
    conv = scn.SubmanifoldConvolution(3, 32, 64, 3, False).to(DEV)
    _lib.set_recorder(rec)
    try:
        y = conv(t).features
        gy = torch.randn_like(y)
        y.backward(gy)
    finally:
        _lib.set_recorder(None)
    # both directions on the per-wave 128-row tiles (msp_conv_tile_form; 32 -> 64 in two 32-column passes)
    assert "subm_fwd/x6r" in rec.kinds and "subm_bwd_data/x6r" in rec.kinds, rec.kinds
    rules = t.metadata.level(4096).subm_rules(3)
    perm, nbp = rules.dense_order()
    y_nbr = ops.conv_nbr(x.detach(), conv.weight.detach().reshape(27, 32, 64).contiguous(), 27, 2, 64, nbp, V,
                         perm=perm)
    nb = rules.nbr.long()
    w = conv.weight.detach().double().reshape(27, 32, 64)  # [K][c_in][c_out]
    x64 = torch.cat([x.detach().double(), torch.zeros(1, 32, dtype=torch.float64, device=DEV)])
    ref = torch.zeros(V, 64, dtype=torch.float64, device=DEV)
    dx = torch.zeros(V + 1, 32, dtype=torch.float64, device=DEV)
    dw = torch.zeros(27, 32, 64, dtype=torch.float64, device=DEV)
    g64 = gy.double()
    for o in range(27):
        src = torch.where(nb[o] >= 0, nb[o], V)
        ref += x64[src] @ w[o]
        dx.index_add_(0, src, g64 @ w[o].t())
        dw[o] = x64[src].t() @ g64
    close(y, ref, 1e-5, "per-wave tiles fwd")
    close(y_nbr, ref, 1e-5, "nbr fwd")
    close(x.grad, dx[:V], 1e-5, "bwd-data")
    close(conv.weight.grad.reshape(27, 32, 64), dw, 1e-5, "dW")


@pytest.mark.parametrize("cin,cout,nbr_form", [(32, 32, False), (64, 32, False), (64, 64, False), (96, 192, False),
                                               (64, 64, True), (96, 96, True)])
def test_weight_layout_flag(cin, cout, nbr_form):
    """flip bit 1 (weights in the module's [K][c_in][c_out] layout, no
    transposed copy) gives bitwise the same output as the [K][c_out][c_in]
    layout, with and without the flip bit, on every 128-row-tile form and on
    msp_conv_nbr; msp_conv_tile rejects any tile height but 128."""
    from sparseconvnet import _lib, ops
    from sparseconvnet._lib import ptr
    torch.manual_seed(cin + 3 * cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    rules = t.metadata.level(64).subm_rules(3)
    V = t.metadata.level(64).n
    x = torch.randn(V, cin, device=DEV)
    w = torch.randn(27, cin, cout, device=DEV) / (27 * cin) ** 0.5  # module layout
    wt = w.transpose(1, 2).contiguous()
    for flip in (0, 1):
        if nbr_form:
            a = ops.conv_nbr(x, wt, 27, flip, cout, rules.nbr, V)
            b = ops.conv_nbr(x, w, 27, flip | 2, cout, rules.nbr, V)
        else:
            a = ops.conv_tile(x, wt, 27, flip, cout, rules, V)
            b = ops.conv_tile(x, w, 27, flip | 2, cout, rules, V)
        assert torch.equal(a, b), (flip, (a - b).abs().max().item())
    tl = rules.tiles_for(64)
    out = torch.empty(V, cout, device=DEV)
    rc = _lib.load().msp_conv_tile(ptr(x), cin, ptr(w), 27, 2, cout, 64, ptr(tl["tile_start"]), ptr(tl["chunk_off"]),
                                   ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), None, 0,
                                   _lib.stream(x.device))
    assert rc != 0 and b"must be 128" in _lib.load().msp_last_error()


@pytest.mark.parametrize("V,C", [(5000, 32), (3001, 64), (777, 36), (1200, 6), (0, 32)])
def test_residual_join_stats(V, C):
    """msp_add_bn_stats: the sum bit-equal to a + b and its partials bit-equal
    to msp_bn_stats on that sum (vector form; C = 6 takes the scalar form)."""
    from sparseconvnet import _lib, ops
    torch.manual_seed(V + C)
    a = torch.randn(V, C, device=DEV) * 2 + 0.5
    b = torch.randn(V, C, device=DEV)
    f, part = ops.ResidualJoinFunction.apply(a, b)
    assert torch.equal(f, a + b)
    ref = ops._bn_partial_buf(V, C, a.device)
    ref.zero_()
    _lib.call("msp_bn_stats", _lib.ptr(a + b), V, C, _lib.ptr(ref), ops._stream(a))
    P = int(_lib.query("msp_bn_partials", _lib.I64(V), C))
    assert torch.equal(part[:P * 2 * C], ref[:P * 2 * C])


@pytest.mark.parametrize("C,leak,nin", [(32, 0.0, False), (64, 0.333, True), (6, 0.0, False)])
def test_residual_block_fused_matches_unfused(C, leak, nin, monkeypatch):
    """ConcatTable(shortcut, BN-SubM-BN-SubM) + AddTable + BN with the fork /
    join fusions against the same modules run one by one with torch adds
    (the unfused composition): outputs, input gradient and every parameter
    gradient bit-equal, running statistics equal.  (The BatchNorm statistics
    epilogues change the fp64 summation order, so they are off here; their own
    comparison is tests/test_gpu_bn_epilogue.py.)"""
    from sparseconvnet import ops
    monkeypatch.setattr(ops, "FUSE_BN_STATS", False)
    torch.manual_seed(C)
    coords, feats = _inputs(3000, 24, n_feat=C)
    g, _ = _pair(coords, feats)
    C2 = C + 16 if nin else C
    def make():
        torch.manual_seed(1)
        blk = scn.Sequential().add(
            scn.ConcatTable().add(scn.NetworkInNetwork(C, C2, False) if nin else scn.Identity()).add(
                scn.Sequential().add(scn.BatchNormLeakyReLU(C, leakiness=leak))
                .add(scn.SubmanifoldConvolution(3, C, C2, 3, False))
                .add(scn.BatchNormLeakyReLU(C2, leakiness=leak))
                .add(scn.SubmanifoldConvolution(3, C2, C2, 3, False)))).add(scn.AddTable()).add(
            scn.BatchNormReLU(C2))
        return blk.to(DEV)
    fused, plain = make(), make()
    def run_plain(x):
        ct, _, bn = list(plain)
        sc, br = list(ct._modules.values())
        a = sc(x)
        y = x
        for m in br:
            y = m(y)
        s = type(x)(a.features + y.features, x.metadata, x.spatial_size)
        return bn(s)
    outs = []
    for run in (fused, run_plain):
        x = g.features.detach().clone().requires_grad_(True)
        t = type(g)(x, g.metadata, g.spatial_size)
        y = run(t)
        w = torch.linspace(-1, 1, y.features.numel(), device=DEV).view_as(y.features)
        (y.features * w).square().sum().backward()
        outs.append((y.features.detach(), x.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    for (n1, p1), (n2, p2) in zip(fused.named_parameters(), plain.named_parameters()):
        assert n1 == n2 and torch.equal(p1.grad, p2.grad), n1
    for (n1, b1), (n2, b2) in zip(fused.named_buffers(), plain.named_buffers()):
        assert torch.equal(b1, b2), n1


@pytest.mark.parametrize("ca,cb,residual", [(32, 32, True), (64, 32, True), (16, 16, False), (6, 10, False)])
def test_join_bn_split_backward_matches_split_pass(ca, cb, residual, monkeypatch):
    """The UNet decoder's JoinTable -> BatchNormalization (residual: the BN fork of ConcatTable(NIN shortcut,
    BN-SubM-BN-SubM) + AddTable; else BN -> SubM): with ops.FUSE_JOIN_SPLIT the BN's backward writes the join
    inputs' gradients as two blocks (msp_bn_bwd_apply_split, ops.BatchNormJoinFunction) instead of a [V][C] dx
    that msp_split_cols then splits.  Outputs, both inputs' gradients, every parameter gradient and the running
    statistics are bit-identical to the split pass (the same arithmetic per element); 6 + 10 channels take the
    scalar kernel.  A second consumer of the joined tensor still gets its gradient through the join."""
    from sparseconvnet import ops
    monkeypatch.setattr(ops, "FUSE_BN_STATS", False)
    torch.manual_seed(ca + 7 * cb)
    coords, feats = _inputs(4000, 24, n_feat=ca)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    C = ca + cb
    b0 = torch.randn(t.features.size(0), cb, device=DEV)

    def make():
        torch.manual_seed(2)
        if residual:
            blk = scn.Sequential().add(scn.JoinTable()).add(
                scn.ConcatTable().add(scn.NetworkInNetwork(C, ca, False)).add(
                    scn.Sequential().add(scn.BatchNormLeakyReLU(C, leakiness=0.333))
                    .add(scn.SubmanifoldConvolution(3, C, ca, 3, False))
                    .add(scn.BatchNormLeakyReLU(ca, leakiness=0.333))
                    .add(scn.SubmanifoldConvolution(3, ca, ca, 3, False)))).add(scn.AddTable())
        else:
            blk = scn.Sequential().add(scn.JoinTable()).add(scn.BatchNormReLU(C)).add(
                scn.SubmanifoldConvolution(3, C, ca, 3, False))
        return blk.to(DEV).train()

    outs = []
    for fuse in (True, False):
        monkeypatch.setattr(ops, "FUSE_JOIN_SPLIT", fuse)
        net = make()
        a = t.features.detach().clone().requires_grad_(True)
        b = b0.clone().requires_grad_(True)
        ta = scn.SparseConvNetTensor(a, t.metadata, t.spatial_size)
        tb = scn.SparseConvNetTensor(b, t.metadata, t.spatial_size)
        y = net([ta, tb]).features
        w = torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)
        (y * w).square().sum().backward()
        outs.append((y.detach(), a.grad, b.grad, [p.grad for p in net.parameters()],
                     [bf.clone() for bf in net.buffers()]))
    for u, v in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(u, v)
    for u, v in zip(outs[0][3] + outs[0][4], outs[1][3] + outs[1][4]):
        assert torch.equal(u, v)
    # a second consumer of the joined tensor: its gradient comes back through the join's split, added to a and b
    monkeypatch.setattr(ops, "FUSE_JOIN_SPLIT", True)
    a = t.features.detach().clone().requires_grad_(True)
    b = b0.clone().requires_grad_(True)
    j = scn.JoinTable().train()([scn.SparseConvNetTensor(a, t.metadata, t.spatial_size),
                                 scn.SparseConvNetTensor(b, t.metadata, t.spatial_size)])
    bn = scn.BatchNormReLU(C).to(DEV).train()
    g1 = torch.randn(a.size(0), C, device=DEV)
    g2 = torch.randn(a.size(0), C, device=DEV)
    ((bn(j).features * g1).sum() + (j.features * g2).sum()).backward()
    ga1, gb1 = a.grad.clone(), b.grad.clone()
    monkeypatch.setattr(ops, "FUSE_JOIN_SPLIT", False)
    a.grad = b.grad = None
    bn2 = scn.BatchNormReLU(C).to(DEV).train()
    j = scn.JoinTable().train()([scn.SparseConvNetTensor(a, t.metadata, t.spatial_size),
                                 scn.SparseConvNetTensor(b, t.metadata, t.spatial_size)])
    ((bn2(j).features * g1).sum() + (j.features * g2).sum()).backward()
    torch.testing.assert_close(ga1, a.grad, rtol=0, atol=1e-6)
    torch.testing.assert_close(gb1, b.grad, rtol=0, atol=1e-6)


@pytest.mark.parametrize("M,K,N", [(300007, 64, 32), (40000, 128, 64), (9001, 192, 96), (5000, 320, 160),
                                   (777, 48, 48), (130, 448, 224), (1, 32, 16), (0, 64, 32), (270001, 32, 64),
                                   (30000, 64, 128), (20000, 96, 192)])
def test_nin_gemm(M, K, N):
    """msp_nin_gemm (NetworkInNetwork forward / backward-data) against an fp64
    product: below 2^18 rows split-bf16 MFMA (the x6 forms' bar, 1e-6 of max
    |ref|), from 2^18 rows fp32 MFMA products and accumulation (1e-5); ragged
    last row group, half-empty last k-slice, one- and two-tile column slices,
    the headline UNet's forward and backward-data shapes."""
    from sparseconvnet import ops
    torch.manual_seed(M + K + N)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV) / K ** 0.5
    out = ops.nin_gemm(a, b)
    assert out.shape == (M, N)
    if M:
        ref = a.double() @ b.double()
        tol = 1e-5 if M >= 1 << 18 else 1e-6
        assert (out.double() - ref).abs().max().item() < tol * ref.abs().max().item()


@pytest.mark.parametrize("M,K,N", [(3001, 40, 24), (500, 8, 20)])
def test_nin_gemm_padded(M, K, N):
    """Channel counts off the 16-grid are zero-padded around msp_nin_gemm."""
    from sparseconvnet import ops
    torch.manual_seed(M)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV)
    ref = a.double() @ b.double()
    assert (ops.nin_gemm(a, b).double() - ref).abs().max().item() < 1e-6 * ref.abs().max().item()


@pytest.mark.parametrize("M,K,N", [(5000, 1200, 64), (3000, 2048, 48), (300000, 1040, 32)])
def test_nin_gemm_deep_k(M, K, N):
    """nIn beyond the kernel's 1024-deep split image (SCN's NetworkInNetwork takes any nIn): 1024-deep slices
    whose products are added in order, on both forms; and a misaligned operand view (odd storage offset)."""
    from sparseconvnet import ops
    torch.manual_seed(M + K)
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV) / K ** 0.5
    ref = a.double() @ b.double()
    tol = 2e-5 if M >= 1 << 18 else 2e-6
    assert (ops.nin_gemm(a, b).double() - ref).abs().max().item() < tol * ref.abs().max().item()
    buf = torch.randn(M * 64 + 1, device=DEV)
    am = buf[1:].view(M, 64)  # 4-byte aligned only
    bm = torch.randn(64, N, device=DEV)
    ref = am.double() @ bm.double()
    assert (ops.nin_gemm(am, bm).double() - ref).abs().max().item() < 1e-5 * ref.abs().max().item()


def test_nin_layer_grad():
    """NetworkInNetwork fwd + bwd (dx via msp_nin_gemm on W^T, dW via msp_conv_wgrad) against fp64 torch."""
    torch.manual_seed(3)
    coords, feats = _inputs(4000, 24, n_feat=64)
    g, _ = _pair(coords, feats)
    nin = scn.NetworkInNetwork(64, 32, False).to(DEV)
    x = g.features.detach().clone().requires_grad_(True)
    y = nin(type(g)(x, g.metadata, g.spatial_size))
    gy = torch.randn_like(y.features)
    y.features.backward(gy)
    xd, wd = x.detach().double(), nin.weight.detach().double()
    close(y.features, xd @ wd, 1e-5, "nin fwd")
    close(x.grad, gy.double() @ wd.t(), 1e-5, "nin dx")
    close(nin.weight.grad, xd.t() @ gy.double(), 1e-5, "nin dW")


def _local_ref(x, wt, nbr, flip):
    V = nbr.size(1)
    x64 = torch.cat([x.double(), torch.zeros(1, x.size(1), dtype=torch.float64, device=DEV)])
    w64 = wt.double().flip(0) if flip else wt.double()
    nb = nbr.long()
    ref = torch.zeros(V, wt.size(1), dtype=torch.float64, device=DEV)
    for o in range(nbr.size(0)):
        ref += x64[torch.where(nb[o] >= 0, nb[o], x.size(0))] @ w64[o].t()
    return ref


def _gather_form(x, wt, flip, cout, rules, V):
    """msp_conv_tile on the 128-row tile rulebook (the gather forms), called directly."""
    from sparseconvnet import _lib
    from sparseconvnet._lib import ptr
    cin = x.size(1)
    tl = rules.tiles_for(128)
    out = torch.empty(V, cout, device=DEV)
    wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(V), 27, cin, cout, 128))
    ws = torch.empty(max(wsb // 4, 1), device=DEV)
    _lib.call("msp_conv_tile", ptr(x), cin, ptr(wt), 27, flip, cout, 128, ptr(tl["tile_start"]),
              ptr(tl["chunk_off"]), ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), ptr(ws), wsb,
              _lib.stream(x.device))
    return out


def _check_local_rulebook(nbr, loc, n):
    K = nbr.size(0)
    T, nt = loc["tile_rows"], loc["n_tiles"]
    us = loc["u_start"][:nt + 1].cpu()
    u_rows = loc["u_rows"].cpu()
    perm = loc["perm"][:nt * T].view(nt, T).cpu()
    lidx = loc["lidx"][:, :nt * T].cpu().to(torch.int64) & 0xFFFF  # uint16 bits in an int16 tensor
    nb = nbr.cpu()
    assert loc["total"] == int(us[-1]) and loc["max_u"] == int((us[1:] - us[:-1]).max())
    for t in range(nt):
        rows = perm[t]
        valid = rows >= 0
        assert int(valid.sum()) == min(T, n - t * T)
        assert bool((~valid[int(valid.sum()):]).all())  # padding last
        assert sorted(rows[valid].tolist()) == list(range(t * T, t * T + int(valid.sum())))
        u = u_rows[int(us[t]):int(us[t + 1])]
        assert bool((u[1:] > u[:-1]).all())
        ent = nb[:, rows[valid].long()]
        assert sorted(set(ent[ent >= 0].tolist())) == u.tolist()
        li = lidx[:, t * T:(t + 1) * T][:, :int(valid.sum())]
        absent = ent < 0
        assert bool((li[absent] == 0xFFFF).all())
        assert torch.equal(u[li[~absent]], ent[~absent])
    wo = loc.get("wave_off")
    if T == 128 and K <= 27:  # conv_x6s's offset lists: per half, every offset some row has, once, packed
        wo = wo[:nt * 64].view(nt, 2, 4, 8).cpu().to(torch.int64)
        has = torch.zeros(K, nt * T, dtype=torch.bool)
        for t in range(nt):
            rows = perm[t]
            has[:, t * T:t * T + int((rows >= 0).sum())] = nb[:, rows[rows >= 0].long()] >= 0
        has = has.view(K, nt, T // 16, 16).any(3)  # [K][tile][group]
        for t in range(nt):
            for h in range(2):
                need = sorted(o for o in range(K) if bool(has[o, t, h::2].any()))
                lists = wo[t, h]
                got = []
                for c in range(4):
                    n = int((lists[c] != 0xFF).sum())
                    assert bool((lists[c, :n] != 0xFF).all()) and bool((lists[c, n:] == 0xFF).all())
                    got += lists[c, :n].tolist()
                assert sorted(got) == need, (t, h)
    else:
        assert wo is None


def test_tile_local_rulebook():
    """msp_tile_local: per 128-row tile the sorted distinct input rows, the rows' order inside the tile
    (by neighbour mask) and the local index of every neighbour, checked entry by entry."""
    from sparseconvnet import _lib, metadata
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    lvl = t.metadata.level(64)
    rules = lvl.subm_rules(3)
    loc = metadata.local_rulebook(rules.nbr, 27, lvl.n, rules.nbr.device, _lib.stream(), 128)
    assert lvl.n % 128 != 0
    _check_local_rulebook(rules.nbr, loc, lvl.n)
    # the rulebook size msp_subm_map_counted wrote beside the map, and the pair lists' count of the same map
    assert rules.n_rules == int((rules.nbr >= 0).sum()) == rules.pairs.total


@pytest.mark.parametrize("n_pts,f", [(1, 3), (1, 5), (7, 3), (300, 5), (5000, 3)])
def test_subm_map_counted_exact_workspace(n_pts, f):
    """msp_subm_map_counted with a workspace of exactly msp_subm_map_workspace_size bytes followed by a canary:
    the kernel's per-block counts stay inside it at every size (the size follows the launch grid; round-5 advice:
    below ~342 rows the old formula was smaller than what the blocks wrote), and the count equals the map's."""
    from sparseconvnet import _lib
    rng = np.random.default_rng(n_pts)
    coords = torch.from_numpy(rng.integers(0, 12, (n_pts, 4)).astype(np.int64))
    coords[:, 3] = 0
    t = scn.InputLayer(3, 16, mode=4)([coords.to(DEV), torch.ones(n_pts, 1, device=DEV)])
    lvl = t.metadata.level(16)
    V = lvl.n
    table, cap = lvl.hash()
    K = f ** 3
    wsb = int(_lib.query("msp_subm_map_workspace_size", _lib.I64(V), f))
    canary = 4096
    buf = torch.full((wsb + canary,), 0xA5, dtype=torch.uint8, device=DEV)
    nbr = torch.empty((K, V), dtype=torch.int32, device=DEV)
    nr = torch.empty(1, dtype=torch.int64, device=DEV)
    _lib.call("msp_subm_map_counted", _lib.ptr(lvl.keys), V, lvl.log2, lvl.size, f, _lib.ptr(table), cap,
              _lib.ptr(nbr), _lib.ptr(nr), _lib.ptr(buf), wsb, _lib.stream())
    torch.cuda.synchronize()
    assert bool((buf[wsb:] == 0xA5).all()), "msp_subm_map_counted wrote past its workspace"
    assert int(nr.item()) == int((nbr >= 0).sum())
    with pytest.raises(RuntimeError, match="workspace too small"):
        _lib.call("msp_subm_map_counted", _lib.ptr(lvl.keys), V, lvl.log2, lvl.size, f, _lib.ptr(table), cap,
                  _lib.ptr(nbr), _lib.ptr(nr), _lib.ptr(buf), wsb - 1, _lib.stream())


@pytest.mark.parametrize("mode", ["random", "dup", "distinct"])
@pytest.mark.parametrize("T,K", [(64, 27), (128, 32), (256, 27)])
def test_tile_local_rulebook_maps(T, K, mode):
    """msp_tile_local's LDS hash-set build on arbitrary maps, every tile size the ABI takes: random rows,
    heavy duplication (5 distinct rows, long probe chains of equal keys) and all K x T entries distinct (the
    largest sort); V not a multiple of T."""
    from sparseconvnet import _lib, metadata
    torch.manual_seed(T + K)
    V = 1000
    if mode == "random":
        nbr = torch.randint(0, 40000, (K, V), dtype=torch.int32, device=DEV)
    elif mode == "dup":
        nbr = torch.randint(0, 5, (K, V), dtype=torch.int32, device=DEV)
    else:
        nbr = (torch.arange(K * V, dtype=torch.int32, device=DEV).view(K, V) * 7919) % (K * V * 2 + 1)
    if mode != "distinct":
        nbr[torch.rand(K, V, device=DEV) < 0.3] = -1
    loc = metadata.local_rulebook(nbr, K, V, nbr.device, _lib.stream(), T)
    _check_local_rulebook(nbr, loc, V)
    if mode == "distinct":
        assert loc["max_u"] == K * T
    # lists only (msp_tile_local with lidx = perm = NULL: what the chunk-local weight gradient reads at level 0)
    lst = metadata.local_rulebook(nbr, K, V, nbr.device, _lib.stream(), T, lists_only=True)
    assert lst["total"] == loc["total"] and lst["max_u"] == loc["max_u"]
    assert torch.equal(lst["u_start"], loc["u_start"]) and torch.equal(lst["u_rows"], loc["u_rows"])


@pytest.mark.parametrize("cin,cout,flip", [(64, 64, 2), (64, 64, 1), (96, 96, 2), (192, 96, 1), (48, 64, 2),
                                           (64, 48, 1), (128, 16, 2), (32, 160, 1)])
def test_conv_local_accuracy(cin, cout, flip):
    """msp_conv_local (tile-local staging, split-bf16 MFMA) against an fp64 evaluation: below 1e-6 of the
    output scale (the x6 forms' bar), and against the production gather form.  flip 2 = forward with the
    module's [K][c_in][c_out] weights, 1 = backward-data ([K][c_out][c_in], offsets mirrored); c_in 48 has a
    half-empty 32-channel slice, c_out 48 / 16 / 160 run one 16-column tile per wave."""
    from sparseconvnet import ops
    torch.manual_seed(cin * 7 + cout + flip)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    lvl = t.metadata.level(64)
    rules = lvl.subm_rules(3)
    V = lvl.n
    x = torch.randn(V, cin, device=DEV)
    w = torch.randn(27, cin, cout, device=DEV) / (27 * cin) ** 0.5
    wt = w if flip == 2 else w.transpose(1, 2).contiguous()
    y = ops.conv_local(x, wt, 27, flip, cout, rules, V)
    ref = _local_ref(x, w.transpose(1, 2), rules.nbr, flip & 1)  # [K][c_out][c_in], offsets mirrored for flip 1
    scale = ref.abs().max().item()
    err = (y.double() - ref).abs().max().item() / scale
    print(f"conv_local {cin}->{cout} flip {flip}: max err {err:.2e} of the output scale")
    assert err < 1e-6, err
    yg = _gather_form(x, wt, flip, cout, rules, V)
    assert (y - yg).abs().max().item() / scale < 2e-6
    # the same rulebook without the offset lists (offsets dealt round-robin to the waves)
    loc = dict(rules.local(), wave_off=None)
    y0 = ops.conv_local(x, wt, 27, flip, cout, type("R", (), {"local": lambda self, tile_rows=128: loc})(), V)
    assert (y0.double() - ref).abs().max().item() / scale < 1e-6


def test_conv_local_overflow_rows():
    """Tiles naming more distinct input rows than the LDS stage holds (383): a random neighbour map over a
    large input (about 1700 distinct rows per tile) sends most rows down the global-memory path; results
    still match fp64, and the metadata is exact."""
    from sparseconvnet import _lib, metadata, ops

    class R:  # a SubmRules stand-in over an arbitrary map
        pass
    torch.manual_seed(5)
    V, n_in, K = 1000, 50000, 27
    nbr = torch.randint(0, n_in, (K, V), dtype=torch.int32, device=DEV)
    nbr[torch.rand(K, V, device=DEV) < 0.5] = -1
    r = R()
    r.nbr, r.K = nbr, K
    loc = metadata.local_rulebook(nbr, K, V, nbr.device, _lib.stream(), 128)
    assert loc["max_u"] > 1000
    _check_local_rulebook(nbr, loc, V)
    r.local = lambda tile_rows=128: loc
    x = torch.randn(n_in, 64, device=DEV)
    w = torch.randn(K, 64, 32, device=DEV) / (K * 64) ** 0.5
    y = ops.conv_local(x, w, K, 2, 32, r, V)
    ref = _local_ref(x, w.transpose(1, 2), nbr, 0)
    assert (y.double() - ref).abs().max().item() / ref.abs().max().item() < 1e-6


@pytest.mark.parametrize("cin,cout", [(32, 32), (64, 32), (32, 64), (96, 64)])
def test_conv_wgrad_chunk_accuracy(cin, cout):
    """msp_conv_wgrad_chunk (chunk-compacted tile-local weight gradient, transposing LDS reads, split-bf16
    MFMA) against an fp64 evaluation of dW[o] = sum_i x[nbr(i, o)]^T dy[i] and against the pair-list form."""
    from sparseconvnet import ops
    torch.manual_seed(cin + 5 * cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    rules = t.metadata.level(64).subm_rules(3)
    V = t.metadata.level(64).n
    x = torch.randn(V, cin, device=DEV)
    dy = torch.randn(V, cout, device=DEV)
    dw = ops.conv_wgrad_chunk(x, dy, rules, 27)
    assert dw is not None
    nb = rules.nbr.long()
    ref = torch.empty(27, cin, cout, dtype=torch.float64, device=DEV)
    for o in range(27):
        m = nb[o] >= 0
        ref[o] = x[nb[o][m]].double().t() @ dy[m].double()
    scale = ref.abs().max().item()
    err = (dw.double() - ref).abs().max().item() / scale
    print(f"wgrad_chunk {cin}x{cout}: max err {err:.2e} of the dW scale")
    assert err < 1e-6
    p = rules.pairs
    dwp = ops.conv_wgrad(x, dy, p, p.pair_in, p.pair_out, 27)
    assert (dw - dwp).abs().max().item() / scale < 2e-6


@pytest.mark.parametrize("cin,cout", [(64, 64), (96, 192)])
def test_conv_wgrad_chunk_from_local_index(cin, cout):
    """The chunk weight gradient's index built from the full tile-local rulebook (msp_local_chunk_index: what
    levels 1-4, whose convolutions take the tile-local form, use since round 5) gives dW within 1e-6 of fp64 and
    of the index built from the 128-row tile rulebook (msp_wgrad_chunk_index), and no tile rulebook is built."""
    from sparseconvnet import metadata, ops
    torch.manual_seed(cin + 7 * cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    rules = t.metadata.level(64).subm_rules(3)
    V = t.metadata.level(64).n
    rules.local()
    assert metadata.LOCAL_CHUNK_INDEX
    idx = rules.wgrad_index(wait=True)
    assert "chunk_src" not in idx["tiles"] and 128 not in rules._tiles and idx["n_far"] == 0
    x = torch.randn(V, cin, device=DEV)
    dy = torch.randn(V, cout, device=DEV)
    dw = ops.conv_wgrad_chunk(x, dy, rules, 27)
    nb = rules.nbr.long()
    ref = torch.empty(27, cin, cout, dtype=torch.float64, device=DEV)
    for o in range(27):
        m = nb[o] >= 0
        ref[o] = x[nb[o][m]].double().t() @ dy[m].double()
    scale = ref.abs().max().item()
    err = (dw.double() - ref).abs().max().item() / scale
    print(f"wgrad_chunk from the local index {cin}x{cout}: max err {err:.2e} of the dW scale")
    assert err < 1e-6
    metadata.LOCAL_CHUNK_INDEX = False
    try:
        rules._wchunk = None
        idx_t = rules.wgrad_index(wait=True)
        assert "chunk_src" in idx_t["tiles"]
        dw_t = ops.conv_wgrad_chunk(x, dy, rules, 27)
    finally:
        metadata.LOCAL_CHUNK_INDEX = True
    assert idx_t["tiles"]["n_chunks"] == idx["tiles"]["n_chunks"]
    assert (dw - dw_t).abs().max().item() / scale < 2e-6


@pytest.mark.parametrize("cin,cout", [(32, 32), (64, 96)])
def test_conv_wgrad_chunk_any_range_count(cin, cout):
    """msp_conv_wgrad_chunk's persistent blocks take contiguous tile ranges of equal cost (chunks + 128 per tile,
    bounds found in-kernel from tile_start) and deal the 27 offsets to their waves by a fitted table (round 6).
    Every range count -- one range, a few, one tile per range, the library's own choice -- gives dW within 1e-5 of
    fp64 (one range keeps every offset's sum in one block's fp32 registers over all tiles: 2.9e-6 measured; the
    library's own count is held to 1e-6 by test_conv_wgrad_chunk_accuracy), each run-to-run bit-identical; and a
    tile count that is not a multiple of the range count is covered."""
    from sparseconvnet import _lib
    from sparseconvnet._lib import ptr
    torch.manual_seed(3 * cin + cout)
    coords, feats = _inputs(20000, 40, n_batch=2)
    t = scn.InputLayer(3, 64, mode=4)([coords.to(DEV), feats.to(DEV)])
    rules = t.metadata.level(64).subm_rules(3)
    V = t.metadata.level(64).n
    idx = rules.wgrad_index(wait=True)
    assert idx["n_far"] == 0
    tiles = idx["tiles"]
    n_tiles = (V + 127) // 128
    x = torch.randn(V, cin, device=DEV)
    dy = torch.randn(V, cout, device=DEV)
    nb = rules.nbr.long()
    ref = torch.empty(27, cin, cout, dtype=torch.float64, device=DEV)
    for o in range(27):
        m = nb[o] >= 0
        ref[o] = x[nb[o][m]].double().t() @ dy[m].double()
    scale = ref.abs().max().item()
    own = int(_lib.query("msp_wgrad_chunk_ranges", _lib.I64(V), cin, cout))
    counts = sorted({1, 3, 7, max(1, n_tiles // 2 + 1), n_tiles, own})
    assert any(n_tiles % c for c in counts)

    def run(n_ranges):
        dw = torch.empty(27, cin, cout, device=DEV)
        slab = torch.empty(n_ranges, 27, cin, cout, device=DEV)
        _lib.call("msp_conv_wgrad_chunk", ptr(x), cin, ptr(dy), cout, 27, tiles["tile_rows"],
                  ptr(tiles["tile_start"]), ptr(tiles["chunk_off"]), ptr(idx["chunk_lr"]), ptr(idx["u_start"]),
                  ptr(idx["u_rows"]), V, n_ranges, ptr(slab), ptr(dw), _lib.stream())
        return dw
    for c in counts:
        a, b = run(c), run(c)
        err = (a.double() - ref).abs().max().item() / scale
        print(f"wgrad_chunk {cin}x{cout} n_tiles={n_tiles} ranges={c}: max err {err:.2e}")
        assert err < (1e-6 if c == own else 1e-5)
        assert torch.equal(a, b)


def test_conv_wgrad_chunk_over_cap_far_rules():
    """A map whose 128-row tiles name more distinct input rows than the chunk weight gradient stages
    (msp_wgrad_chunk_cap, 448): msp_wgrad_chunk_index counts the rules whose row lies past the cap (n_far, ADVICE
    r02: no silent loss at the C ABI), msp_wgrad_far_list lists exactly those, sorted by (offset, entry), and the
    module's backward -- the chunk form plus msp_conv_wgrad_far for the listed rules -- matches fp64."""
    from sparseconvnet import _lib, metadata, ops
    from sparseconvnet._lib import ptr
    torch.manual_seed(9)
    V, K = 20000, 27  # the module's backward asks for the chunk form first (c_out = 64)
    # the SubmRules machinery over this map (square: inputs are rows of the same level), through a stand-in
    r = metadata.SubmRules.__new__(metadata.SubmRules)
    r._plan, r._key, r.K, r.filter_size = [], ("subm", 0, 3), K, 3
    r.nbr = torch.randint(0, V, (K, V), dtype=torch.int32, device=DEV)
    r.nbr[torch.rand(K, V, device=DEV) < 0.2] = -1
    r.nbr[13] = torch.arange(V, dtype=torch.int32, device=DEV)  # the centre offset
    r._tiles, r._locals, r._wchunk, r._dense = {}, {}, None, None
    r._map, r._n = r.nbr, V
    r._pairs = metadata.PairLists(r.nbr, K, V, DEV, _lib.stream(), r._plan, r._key)
    r._n_rules = int((r.nbr >= 0).sum())
    loc = r.local()
    cap = int(_lib.query("msp_wgrad_chunk_cap"))
    assert loc["max_u"] > cap  # random rows: ~27 x 0.8 x 128 per tile
    idx = r.wgrad_index()
    assert idx is not None and idx["n_far"] > 0
    # the C ABI: the over-cap rules are counted, not silently dropped, and the list names exactly them
    tiles = r.tiles_for(128)
    lr = torch.empty(tiles["n_chunks"] * 16, dtype=torch.int32, device=DEV)
    n_far = torch.full((1,), -1, dtype=torch.int64, device=DEV)
    _lib.call("msp_wgrad_chunk_index", ptr(tiles["tile_start"]), ptr(tiles["chunk_src"]), ptr(tiles["chunk_row"]),
              _lib.I64(V), ptr(loc["u_start"]), ptr(loc["u_rows"]), ptr(lr), ptr(n_far), _lib.stream())
    u = loc["u_start"][:loc["n_tiles"] + 1].cpu()
    assert int(n_far.item()) == idx["n_far"] and bool(((u[1:] - u[:-1]) > cap).any())
    w_lr = lr.cpu().long() & 0xFFFFFFFF
    far_e = torch.nonzero(((w_lr & 0xFFFF) == 0xFFFF) & ((w_lr >> 16) < 128)).flatten()
    off = tiles["chunk_off"].cpu().long()[far_e // 16]
    want = torch.sort((off << 40) | far_e).values
    assert torch.equal(idx["far_key"].cpu(), want)
    ts = tiles["tile_start"].cpu()
    assert torch.equal(idx["far_tile"].cpu().long(), torch.searchsorted(ts[1:loc["n_tiles"] + 1], (want & ((1 << 40) - 1)) // 16, right=True))
    # the weight gradient through the autograd Function
    assert int(_lib.query("msp_wgrad_chunk_preferred", _lib.I64(V), K, 32, 64))
    x = torch.randn(V, 32, device=DEV, requires_grad=True)
    w = (torch.randn(K, 1, 32, 64, device=DEV) / (K * 32) ** 0.5).requires_grad_(True)
    y = ops.SubmanifoldConvFunction.apply(x, w, r)
    dy = torch.randn_like(y)
    y.backward(dy)
    nb = r.nbr.long()
    ref = torch.empty(K, 32, 64, dtype=torch.float64, device=DEV)
    for o in range(K):
        m = nb[o] >= 0
        ref[o] = x.detach().double()[nb[o][m]].t() @ dy.double()[m]
    dw = w.grad.reshape(K, 32, 64).double()
    assert (dw - ref).abs().max().item() / ref.abs().max().item() < 1e-6


@pytest.mark.parametrize("n,end_bit,span", [(1, 8, 256), (4095, 12, 3000), (4097, 39, 1 << 39), (300001, 39, 5000),
                                            (1600000, 39, 1 << 39), (70000, 64, 0), (5000, 20, 7)])
def test_sort_pairs_stable(n, end_bit, span):
    """msp_sort_pairs (the library's own LSD radix sort: ballot-ranked scatter, msp_sort.hip) against numpy's
    stable argsort on key bits [0, end_bit): ragged last tiles, one-digit and five-digit sorts, heavy duplicates
    (stability decides the values' order), all-ones keys (the InputLayer's out-of-range sentinel) and a 64-bit
    sort of full-range keys."""
    import numpy as np
    from sparseconvnet import _lib
    from sparseconvnet._lib import ptr
    rng = np.random.default_rng(n + end_bit)
    if span:
        keys = rng.integers(0, span, n, dtype=np.uint64)
    else:
        keys = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    keys[rng.random(n) < 0.01] = np.uint64(0xFFFFFFFFFFFFFFFF)
    masked = keys & np.uint64((1 << end_bit) - 1) if end_bit < 64 else keys
    order = np.argsort(masked, kind="stable")
    kin = torch.from_numpy(keys.view(np.int64)).to(DEV)
    vin = torch.arange(n, dtype=torch.int32, device=DEV)
    kout, vout = torch.empty_like(kin), torch.empty_like(vin)
    wsb = int(_lib.query("msp_sort_workspace_size", n, end_bit))
    ws = torch.empty(wsb, dtype=torch.uint8, device=DEV)
    _lib.call("msp_sort_pairs", ptr(kin), ptr(kout), ptr(vin), ptr(vout), n, end_bit, ptr(ws), wsb, _lib.stream())
    assert np.array_equal(vout.cpu().numpy(), order.astype(np.int32))
    assert np.array_equal(kout.cpu().numpy().view(np.uint64), keys[order])
