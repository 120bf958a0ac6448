"""End-to-end parity of the registered encoders (HIP path vs CPU oracle, fp64).

The bar from BASELINE.json's north star: per-point outputs within 1e-4 of the
reference path (fp32): max|gpu - oracle| <= 1e-4 * max(1, max|oracle|) on the
per-point features and the scene features.

Gradients: the oracle runs with the device's ReLU sign decisions
(oracle/parity.py) -- two valid fp32 evaluations may put a BatchNorm output
that is within rounding of 0 on different sides, which changes that
element's gradient by O(|dy|).  With shared decisions every parameter
gradient must match to 1e-4 of its tensor's max; the number of decisions the
fp64 oracle would have taken differently is reported and each must sit at
rounding level (|z| < 1e-4).  Parameter gradients must then match to 1e-3 of
each tensor's max: the oracle itself evaluated in fp32 (same code, CPU)
differs from its fp64 run by up to 2.3e-4 on these tensors (median 1.3e-5),
so 1e-3 is the fp32 envelope, while an indexing or formula error shows up at
O(1).
"""
import pytest
import torch

import sparseconvnet as scn  # noqa: F401
from oracle.encoders import OracleEncoder
from oracle.parity import run_shared_masks
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CASES = [
    # name, m, reps, residual, scale, scenes, spacing
    ("SparseConvUNet", 16, 1, False, 12, 2, 0.04),          # C2 shape, reduced
    ("SparseConvUNet", 32, 2, True, 10, 1, 0.05),           # C3 shape (headline), reduced
    ("SparseConvFCNet", 16, 1, False, 10, 1, 0.05),          # C5 / C1 family
    ("SparseConvFCNetEncoder", 16, 1, False, 10, 1, 0.05),   # C1
    ("SparseConvFCNetDirectUpPool", 16, 1, True, 10, 1, 0.05),
    ("SparseConvFCNetDirectUpPoolLight", 16, 1, False, 10, 1, 0.05),  # stride-4 path
]


def _models(name, m, reps, residual, scale, scenes, spacing):
    torch.manual_seed(7)
    batch = make_batch(scenes, scale, seed=11, spacing=spacing)
    cfg = dict(m=m, dimension=3, full_scale=4096, block_reps=reps, residual_blocks=residual)
    cls, _ = MODEL_REGISTRY.get(name)
    model = cls(name, **cfg).to(DEV)
    ref = OracleEncoder(name, **cfg).double()
    res = ref.load_state_dict({k: v.double().cpu() for k, v in model.state_dict().items()})
    assert not res.missing_keys and not res.unexpected_keys
    coords = torch.from_numpy(batch["coords"])
    feats = torch.from_numpy(batch["feats"])
    xg = EasyDict(coords=coords.to(DEV), feature=feats.to(DEV), batch_offsets=batch["batch_offsets"])
    xo = dict(coords=coords, feature=feats.double(), batch_offsets=batch["batch_offsets"])
    return model, ref, xg, xo


def _close(a, b, tol, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = (a - b).abs().max().item()
    lim = tol * max(1.0, b.abs().max().item())
    assert err <= lim, f"{what}: {err:.3e} > {lim:.3e}"
    return err


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-m{c[1]}-r{c[2]}" for c in CASES])
def test_encoder_train_parity(case):
    model, ref, xg, xo = _models(*case)
    # per-point features (eval of the same batch statistics: train-mode forward)
    out_g, out_o, _ = run_shared_masks(model, ref, xg, xo, istrain=False)
    _close(out_g, out_o, 1e-4, "per-point features")
    glob_g, glob_o, st = run_shared_masks(model, ref, xg, xo, istrain=True)
    _close(glob_g, glob_o, 1e-4, "scene features")
    assert st["max_flip_margin"] < 1e-4, st
    w = torch.linspace(-1, 1, glob_o.shape[1], dtype=torch.float64)
    (glob_g * w.float().to(DEV)).sum().backward()
    (glob_o * w).sum().backward()
    gg = dict(model.named_parameters())
    for k, p in ref.named_parameters():
        g_gpu = gg[k].grad
        assert g_gpu is not None, k
        scale = max(p.grad.abs().max().item(), 1e-12)
        err = (g_gpu.double().cpu() - p.grad).abs().max().item()
        assert err <= 1e-3 * scale + 1e-9, f"grad {k}: {err:.3e} vs scale {scale:.3e} ({st})"


@pytest.mark.parametrize("case", CASES[:2], ids=["unet-m16", "unet-m32-res"])
def test_encoder_eval_parity(case):
    model, ref, xg, xo = _models(*case)
    model.eval()
    ref.eval()
    out_g, out_o, _ = run_shared_masks(model, ref, xg, xo, istrain=False)
    _close(out_g, out_o, 1e-4, "eval per-point features")
    # and independently of the shared decisions
    with torch.no_grad():
        _close(model(xg), ref(xo), 1e-4, "eval per-point features (free run)")


def test_free_run_forward_parity():
    """Without shared ReLU decisions the headline-shaped UNet still meets the
    1e-4 per-point bar in train mode."""
    model, ref, xg, xo = _models(*CASES[1])
    _close(model(xg), ref(xo), 1e-4, "per-point features (free run)")


def test_counters_match_oracle():
    import oracle.scn_oracle as O
    model, ref, xg, xo = _models(*CASES[0])
    scn.forward_pass_multiplyAdd_count = 0
    scn.forward_pass_hidden_states = 0
    O.forward_pass_multiplyAdd_count = 0
    O.forward_pass_hidden_states = 0
    model(xg)
    ref(xo)
    assert scn.forward_pass_multiplyAdd_count == O.forward_pass_multiplyAdd_count > 0
    assert scn.forward_pass_hidden_states == O.forward_pass_hidden_states > 0


@pytest.mark.parametrize("name,m", [("SparseConvUNet", 16), ("SparseConvFCNet", 8)])
def test_fused_scene_mean_matches_per_point_path(name, m):
    """istrain=True runs the fused tail (scene means from the voxel rows, no
    (N, C) per-point tensor); it must equal OutputLayer + per-scene torch.mean
    (models/SparseConvNet.py:20-26) in value and in every parameter gradient,
    and a batch whose ranges do not match the batch column falls back to the
    per-point path."""
    torch.manual_seed(3)
    batch = make_batch(3, 10, seed=5, spacing=0.05)
    cfg = dict(m=m, dimension=3, full_scale=4096, block_reps=1, residual_blocks=False)
    cls, _ = MODEL_REGISTRY.get(name)
    model = cls(name, **cfg).to(DEV)
    assert model._fusable()
    x = EasyDict(coords=torch.from_numpy(batch["coords"]).to(DEV), feature=torch.from_numpy(batch["feats"]).to(DEV),
                 batch_offsets=batch["batch_offsets"])
    w = torch.randn(3, model(x).size(1), device=DEV)

    def run(fused):
        model.zero_grad()
        if fused:
            out = model(x, istrain=True)
        else:
            from wsss3d.encoders import segment_mean
            out = segment_mean(model(x), x.batch_offsets)
        (out * w).square().sum().backward()
        return out.detach(), {k: p.grad.detach().clone() for k, p in model.named_parameters()}

    of, gf = run(True)
    op, gp = run(False)
    _close(of, op, 1e-5, "scene means")
    for k in gp:
        _close(gf[k], gp[k], 1e-4, "grad " + k)
    # batch column not matching the ranges: the fused path must not be taken
    xb = EasyDict(coords=x.coords.clone(), feature=x.feature, batch_offsets=x.batch_offsets)
    xb.coords[0, -1] = 2
    with torch.no_grad():
        outb = model(xb, istrain=True)
        from wsss3d.encoders import segment_mean
        refb = segment_mean(model(xb), xb.batch_offsets)
    _close(outb, refb, 1e-6, "fallback")


def test_metadata_prefetch_matches_inline():
    """sparseconvnet.prefetch_metadata (side-stream build of the next batch's
    voxelisation and every rulebook the last forward requested) gives bitwise
    the same logits and parameter gradients as building it inside the
    forward, and the prefetched forward records the same plan."""
    import sparseconvnet as scn
    from wsss3d import EasyDict, MODEL_REGISTRY
    from wsss3d.synthetic import make_batch
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("SparseConvUNet")
    model = cls("SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True).cuda()
    bs = [make_batch(2, 20, seed=s) for s in (11, 12)]
    xs = [EasyDict(coords=torch.from_numpy(b["coords"]).cuda(), feature=torch.from_numpy(b["feats"]).cuda(),
                   batch_offsets=b["batch_offsets"]) for b in bs]

    def run(x):
        model.zero_grad(set_to_none=True)
        out = model(x)
        out.square().sum().backward()
        return out.detach().clone(), [p.grad.clone() for p in model.parameters()]

    run(xs[0])                      # records the plan
    ref_out, ref_g = run(xs[1])     # inline build
    plan = list(model.encoder[0].last_plan)
    assert any(e[0] == "down" for e in plan) and any(e[0] == "subm" for e in plan)
    m = scn.prefetch_metadata(model, xs[1].coords)
    assert m is not None
    out, g = run(xs[1])             # consumes the prefetched metadata
    assert model.encoder[0].last_plan is m.plan
    assert torch.equal(out, ref_out)
    for a, b in zip(g, ref_g):
        assert torch.equal(a, b)


def test_prefetch_batches_count_reads():
    """A replay reads its rulebook counts together (metadata._Deferred): the prefetch synchronises the host
    with the device twice for the voxelisation, once per coarsening and once at the end, and every rulebook it
    built -- tile, tile-local and pair-list counts -- equals the one an inline build of the same batch makes."""
    import warnings
    from sparseconvnet import metadata as md
    from wsss3d import EasyDict
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("SparseConvUNet")
    model = cls("SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True).to(DEV)
    bs = [make_batch(2, 20, seed=s) for s in (31, 32)]
    xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                   batch_offsets=b["batch_offsets"]) for b in bs]
    model(xs[0]).square().sum().backward()    # records the plan (forward and backward uses)
    inline = md.Metadata(DEV)
    inline.build_input(xs[1].coords, 4096)
    plan = list(model.encoder[0].last_plan)
    n_down = sum(1 for e in plan if e[0] == "down")
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            m = md.Metadata(DEV)
            m.build_input(xs[1].coords, 4096)
            n_input = len(w)
            m.replay(plan)
            n_replay = len(w) - n_input
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert n_replay <= n_down + 1, (n_replay, n_down)
    for e in plan:   # the inline build: the same levels, each count read where it is taken
        if e[0] == "down":
            inline.downsample(e[1], e[2])
        elif e[0] == "subm":
            inline.level(e[1]).subm_rules(e[2])
    for size, lvl in m.levels.items():
        ref = inline.levels[size]
        assert lvl.n == ref.n and torch.equal(lvl.keys, ref.keys)
        for fs, r in lvl.subm.items():
            q = ref.subm[fs]
            assert r.n_rules == q.n_rules and r.pairs.counts == q.pairs.counts
            for tr, t in r._tiles.items():
                u = q.tiles_for(tr)
                assert t["n_chunks"] == u["n_chunks"] and t["max_chunks"] == u["max_chunks"]
                for k in ("tile_start", "chunk_off", "chunk_src", "chunk_row"):
                    assert torch.equal(t[k][:u[k].numel()], u[k]), (size, tr, k)
            for tr, t in r._locals.items():
                u = q.local(tr)
                assert (t["total"], t["max_u"]) == (u["total"], u["max_u"])
                for k in ("u_start", "u_rows", "lidx", "perm"):
                    assert torch.equal(t[k], u[k]), (size, tr, k)
            if r.pairs._pin is not None:
                assert torch.equal(r.pairs.pair_in, q.pairs.pair_in)
                assert torch.equal(r.pairs.pair_out, q.pairs.pair_out)
            if r._wchunk:
                wq = q.wgrad_index(wait=True)
                assert wq is not None and torch.equal(r._wchunk["chunk_lr"], wq["chunk_lr"])
                assert r._wchunk["n_far"] == wq["n_far"]  # rules past a tile's staged rows, counted in the replay
                if wq["n_far"]:
                    assert torch.equal(r._wchunk["far_key"], wq["far_key"])
        for stride, (csize, r) in lvl.down.items():
            q = ref.down[stride][1]
            assert r.pairs.counts == q.pairs.counts and torch.equal(r.down, q.down)


def _prefetch_model():
    from wsss3d import EasyDict
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("MultiLabel")
    pc = EasyDict(name="SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True)
    model = cls(pc).to(DEV)
    bs = [make_batch(2, 20, seed=s) for s in (21, 22)]
    xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                   batch_offsets=b["batch_offsets"]) for b in bs]
    ys = [torch.from_numpy(b["scene_labels"]).to(DEV) for b in bs]
    return model, xs, ys


def test_prefetched_step_has_no_host_read():
    """A training step whose metadata was prefetched (the bench loop: forward with the fused tail, loss,
    backward, fused Adam) issues no device-to-host read or synchronising copy: torch's sync debug mode
    raises on any (.item(), .tolist(), blocking copies)."""
    import torch.nn.functional as F
    model, xs, ys = _prefetch_model()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)

    def step(k):
        opt.zero_grad(set_to_none=True)
        logits, _ = model((xs[k], None), istrain=True)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    step(0)                                   # records the plan, builds the optimizer state
    torch.cuda.synchronize()
    assert scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False) is not None
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        step(1)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in model.parameters())


def test_prefetch_entry_needs_the_same_tensor():
    """The prefetched entry is found only through the very coords tensor it was built for (a copy at
    another address, or a new tensor at a reused address, builds its own metadata), and a newer prefetch
    drops an unconsumed older one."""
    from sparseconvnet import metadata as md
    model, xs, _ = _prefetch_model()
    with torch.no_grad():
        model(xs[0])                           # records the plan
        m = scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False)
        twin = xs[1].coords.clone()
        assert md.take_prefetched(twin, 4096) is None
        assert md.pending_count() == 1         # still pending for the original tensor
        m2 = scn.prefetch_metadata(model, xs[0].coords, wait_for_producer=False)
        assert md.pending_count() == 1         # the older entry was dropped
        assert md.take_prefetched(xs[1].coords, 4096) is None
        assert md.take_prefetched(xs[0].coords, 4096) is m2 and m2 is not m
        assert md.pending_count() == 0
        # depth 2 (bench.py --prefetch-thread): two batches pending at once, each found through its own tensor,
        # a third drops the oldest, and the same tensor again replaces its own entry
        md.PREFETCH_DEPTH = 2
        try:
            a = scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False)
            b = scn.prefetch_metadata(model, xs[0].coords, wait_for_producer=False)
            assert md.pending_count() == 2 and md.prefetch_event(DEV, xs[1].coords) is not None
            b2 = scn.prefetch_metadata(model, xs[0].coords, wait_for_producer=False)
            assert md.pending_count() == 2 and b2 is not b
            c = scn.prefetch_metadata(model, twin, wait_for_producer=False)
            assert md.pending_count() == 2 and md.take_prefetched(xs[1].coords, 4096) is None   # a was dropped
            assert md.take_prefetched(twin, 4096) is c and md.take_prefetched(xs[0].coords, 4096) is b2
            assert md.pending_count() == 0 and a is not None
        finally:
            md.PREFETCH_DEPTH = 1


def test_graph_captured_step_matches_eager():
    """bench.py --graph: a training step captured into a HIP graph after its metadata was prefetched, then
    replayed, leaves parameters, gradients and Adam state bit-identical to the same step launched eagerly
    (same kernels in the same order), and the capture consumes the prefetched metadata."""
    import copy
    import torch.nn.functional as F
    from sparseconvnet import metadata as md
    model, xs, ys = _prefetch_model()
    twin = copy.deepcopy(model)
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True) for m in (model, twin)]

    def body(m, opt, k):
        opt.zero_grad(set_to_none=True)
        logits, _ = m((xs[k], None), istrain=True)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    for m, opt in zip((model, twin), opts):   # plan + optimizer state, eagerly
        body(m, opt, 0)
    torch.cuda.synchronize()
    scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False)
    body(model, opts[0], 1)                   # eager, prefetched
    scn.prefetch_metadata(twin, xs[1].coords, wait_for_producer=False)
    ev = md.prefetch_event(DEV)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        g.capture_begin()
        body(twin, opts[1], 1)
        g.capture_end()
    keep = md.captured_metadata()
    assert len(keep) == 1 and md.pending_count() == 0
    cur = torch.cuda.current_stream()
    cur.wait_event(ev)
    g.replay()
    torch.cuda.synchronize()
    for (na, a), (nb, b) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(a, b), na
        assert torch.equal(a.grad, b.grad), na
    for sa, sb in zip(opts[0].state.values(), opts[1].state.values()):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k], sb[k])


@pytest.mark.parametrize("where", ["forward", "backward"])
def test_capture_error_is_a_clean_error(where):
    """An error raised inside a captured step (a module whose forward raises; a gradient hook that raises in
    backward) comes out of sparseconvnet.graphs.capture as that RuntimeError, with the capture ended and the
    graph discarded -- not an abort of the process (round-5 verdict: ~CUDAGraph on an open capture called
    std::terminate).  The process then runs an eager step, and a captured + replayed step, bit-identical to a
    twin model that never saw the failed capture (weight images on, so the discarded prepare() must not be
    trusted)."""
    import copy
    import torch.nn.functional as F
    from sparseconvnet import metadata as md
    model, xs, ys = _prefetch_model()
    twin = copy.deepcopy(model)
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True) for m in (model, twin)]
    wimg = scn.weight_images.enable(twin, DEV, optimizer=opts[1])
    fail = [False]

    def boom(*_):
        if fail[0]:
            raise RuntimeError("injected failure inside the capture")

    enc = twin.pc_encoder.encoder
    hook = list(enc)[2].register_forward_hook(boom) if where == "forward" else None

    def body(m, opt, k, images=None):
        if images is not None:
            images.prepare()
        opt.zero_grad(set_to_none=True)
        logits, _ = m((xs[k], None), istrain=True)
        if where == "backward" and m is twin:
            logits.register_hook(lambda g: boom() or g)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    try:
        for m, opt in zip((model, twin), opts):   # plan, optimizer state and image descriptors, eagerly
            body(m, opt, 0, wimg if m is twin else None)
        wimg.build()
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        scn.prefetch_metadata(twin, xs[1].coords, wait_for_producer=False)
        fail[0] = True
        with pytest.raises(RuntimeError, match="injected failure"):
            scn.graphs.capture(lambda: body(twin, opts[1], 1, wimg), side)
        fail[0] = False
        assert not torch.cuda.is_current_stream_capturing()
        assert md.captured_metadata() == [] and md.pending_count() == 0
        assert not wimg.valid  # the discarded capture's prepare() is not trusted
        # an eager step on both, then a captured + replayed step on the twin against an eager one
        body(model, opts[0], 1)
        body(twin, opts[1], 1, wimg)
        scn.prefetch_metadata(model, xs[0].coords, wait_for_producer=False)
        body(model, opts[0], 0)
        wimg.build()
        scn.prefetch_metadata(twin, xs[0].coords, wait_for_producer=False)
        ev = md.prefetch_event(DEV)
        g, _ = scn.graphs.capture(lambda: body(twin, opts[1], 0, wimg), side)
        keep = md.captured_metadata()
        assert len(keep) == 1
        torch.cuda.current_stream().wait_event(ev)
        g.replay()
        torch.cuda.synchronize()
    finally:
        scn.weight_images.disable()
        if hook is not None:
            hook.remove()
    for (na, a), (nb, b) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(a, b), na
        assert torch.equal(a.grad, b.grad), na
    for sa, sb in zip(opts[0].state.values(), opts[1].state.values()):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k], sb[k])


def test_graph_capture_beside_worker_prefetch():
    """bench.py --prefetch-thread: each step is captured while a worker thread builds the metadata of the next
    batch on the side stream (two prefetched batches pending, PREFETCH_DEPTH = 2); three captured and replayed
    steps leave parameters, gradients and Adam state bit-identical to the same steps launched eagerly."""
    import copy
    from concurrent.futures import ThreadPoolExecutor
    import torch.nn.functional as F
    from sparseconvnet import metadata as md
    model, xs, ys = _prefetch_model()
    twin = copy.deepcopy(model)
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True) for m in (model, twin)]

    def body(m, opt, k):
        opt.zero_grad(set_to_none=True)
        logits, _ = m((xs[k], None), istrain=True)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    for m, opt in zip((model, twin), opts):   # plan + optimizer state, eagerly
        body(m, opt, 0)
    torch.cuda.synchronize()
    seq = [1, 0, 1]
    for k in seq:                             # eager reference, prefetched on the loop's thread
        scn.prefetch_metadata(model, xs[k].coords, wait_for_producer=False)
        body(model, opts[0], k)
    torch.cuda.synchronize()
    md.PREFETCH_DEPTH = 2
    pool = ThreadPoolExecutor(max_workers=1)
    graphs, keeps = [], []
    try:
        scn.prefetch_metadata(twin, xs[seq[0]].coords, wait_for_producer=False)
        fut = pool.submit(scn.prefetch_metadata, twin, xs[seq[1]].coords, False)
        side = torch.cuda.Stream()
        cur = torch.cuda.current_stream()
        for j, k in enumerate(seq):
            ev = md.prefetch_event(DEV, xs[k].coords)
            assert ev is not None
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                g.capture_begin(capture_error_mode="relaxed")
                body(twin, opts[1], k)
                g.capture_end()
            keeps.append(md.captured_metadata())
            assert len(keeps[-1]) == 1
            cur.wait_event(ev)
            g.replay()
            graphs.append(g)
            if fut is not None:
                fut.result()
                fut = pool.submit(scn.prefetch_metadata, twin, xs[seq[j + 2]].coords, False) \
                    if j + 2 < len(seq) else None
        torch.cuda.synchronize()
    finally:
        pool.shutdown()
        md.PREFETCH_DEPTH = 1
    assert md.pending_count() == 0
    for (na, a), (nb, b) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(a, b), na
        assert torch.equal(a.grad, b.grad), na
    for sa, sb in zip(opts[0].state.values(), opts[1].state.values()):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k], sb[k])


def test_graph_capture_after_a_smaller_batch():
    """The prefetched plan comes from the previous batch, whose level sizes may select other rulebooks (the
    tile-local form from 4096 rows at 64 channels): replay
    prepares what THIS batch's sizes select (recorded uses, ops.prepare), so a capture after a much smaller
    batch builds nothing on demand (a host read there would abort the capture), and it matches eager."""
    import copy
    import torch.nn.functional as F
    from sparseconvnet import metadata as md
    from wsss3d import EasyDict
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("MultiLabel")
    pc = EasyDict(name="SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True)
    model = cls(pc).to(DEV)
    twin = copy.deepcopy(model)
    bs = [make_batch(1, 12, seed=31), make_batch(4, 50, seed=32)]
    xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                   batch_offsets=b["batch_offsets"]) for b in bs]
    ys = [torch.from_numpy(b["scene_labels"]).to(DEV) for b in bs]
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True) for m in (model, twin)]

    def body(m, opt, k):
        opt.zero_grad(set_to_none=True)
        logits, _ = m((xs[k], None), istrain=True)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    for m, opt in zip((model, twin), opts):   # the small batch, eagerly: its plan
        body(m, opt, 0)
    torch.cuda.synchronize()
    scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False)
    body(model, opts[0], 1)
    scn.prefetch_metadata(twin, xs[1].coords, wait_for_producer=False)
    ev = md.prefetch_event(DEV)
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        g.capture_begin(capture_error_mode="relaxed")
        body(twin, opts[1], 1)
        g.capture_end()
    md.captured_metadata()
    torch.cuda.current_stream().wait_event(ev)
    g.replay()
    torch.cuda.synchronize()
    for (na, a), (nb, b) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(a, b), na
        assert torch.equal(a.grad, b.grad), na
