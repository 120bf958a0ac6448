"""Per-step split-weight images (sparseconvnet.weight_images, include/mi3dsparse.h msp_weight_image): training
steps whose convolutions take the images prepared in one launch at the step start leave parameters, gradients and
Adam state bit-identical to steps whose every call splits its own, eagerly and inside a HIP graph capture; an
image whose weights changed after it was prepared is never used."""
import copy

import pytest
import torch
import torch.nn.functional as F

import sparseconvnet as scn
from wsss3d import EasyDict, MODEL_REGISTRY
from wsss3d.synthetic import make_batch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _model():
    torch.manual_seed(0)
    cls, _ = MODEL_REGISTRY.get("MultiLabel")
    # m = 32 at 2 cm: per-wave tiles (level 0), tile-local (levels 1-3), dense groups (level 0's 32 -> 64
    # backward-data) and shared tiles (the small levels) all take images
    pc = EasyDict(name="SparseConvUNet", m=32, dimension=3, full_scale=4096, block_reps=1, residual_blocks=True)
    model = cls(pc).to(DEV)
    bs = [make_batch(2, 50, seed=s) for s in (41, 42)]
    xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(DEV), feature=torch.from_numpy(b["feats"]).to(DEV),
                   batch_offsets=b["batch_offsets"]) for b in bs]
    ys = [torch.from_numpy(b["scene_labels"]).to(DEV) for b in bs]
    return model, xs, ys


def _same(model, twin, opts):
    for (na, a), (nb, b) in zip(model.named_parameters(), twin.named_parameters()):
        assert torch.equal(a, b), na
        assert torch.equal(a.grad, b.grad), na
    for sa, sb in zip(opts[0].state.values(), opts[1].state.values()):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k], sb[k])


def test_weight_images_match_per_call_splits():
    model, xs, ys = _model()
    twin = copy.deepcopy(model)
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True) for m in (model, twin)]
    images = scn.weight_images.enable(model, optimizer=opts[0])
    try:
        for k in range(4):
            for m, opt, wi in ((model, opts[0], images), (twin, opts[1], None)):
                if wi is not None:
                    wi.prepare()
                    scn.weight_images._ACTIVE = wi
                else:
                    scn.weight_images._ACTIVE = None
                opt.zero_grad(set_to_none=True)
                logits, _ = m((xs[k % 2], None), istrain=True)
                F.multilabel_soft_margin_loss(logits, ys[k % 2]).backward()
                opt.step()
        torch.cuda.synchronize()
        assert len(images.entries) >= 10 and images.hits >= 10, (len(images.entries), images.hits)
        _same(model, twin, opts)
    finally:
        scn.weight_images.disable()


def test_stale_image_is_not_used():
    """A change of the weights after prepare() -- an optimizer step (fused Adam bumps no version counter: the
    step post-hook catches it) or an in-place update -- makes every call split its own again until the next
    prepare()."""
    model, xs, ys = _model()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    images = scn.weight_images.enable(model, optimizer=opt)
    try:
        for k in range(2):
            images.prepare()
            opt.zero_grad(set_to_none=True)
            logits, _ = model((xs[k % 2], None), istrain=True)
            F.multilabel_soft_margin_loss(logits, ys[k % 2]).backward()
            opt.step()
        h = images.hits
        assert h > 0
        logits, _ = model((xs[0], None), istrain=True)  # weights changed since the last prepare(): no image
        assert images.hits == h
        images.prepare()
        logits, _ = model((xs[0], None), istrain=True)
        assert images.hits > h
        h = images.hits
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.0)  # in-place changes: version counters bumped
        model((xs[0], None), istrain=True)
        assert images.hits == h
    finally:
        scn.weight_images.disable()


def test_weight_images_in_a_captured_step():
    """The bench's graph mode: prepare() and the convolutions captured into one HIP graph, replayed: identical
    to the same step launched eagerly with per-call splits."""
    from sparseconvnet import metadata as md
    model, xs, ys = _model()
    twin = copy.deepcopy(model)
    opts = [torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True) for m in (model, twin)]
    images = scn.weight_images.enable(twin, optimizer=opts[1])

    def body(m, opt, k, wi):
        scn.weight_images._ACTIVE = wi
        if wi is not None:
            wi.prepare()
        opt.zero_grad(set_to_none=True)
        logits, _ = m((xs[k], None), istrain=True)
        F.multilabel_soft_margin_loss(logits, ys[k]).backward()
        opt.step()

    try:
        body(model, opts[0], 0, None)
        body(twin, opts[1], 0, images)      # records the descriptors
        torch.cuda.synchronize()
        images.build()
        scn.weight_images._ACTIVE = None
        scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False)
        body(model, opts[0], 1, None)
        scn.prefetch_metadata(twin, xs[1].coords, wait_for_producer=False)
        ev = md.prefetch_event(DEV)
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        h = images.hits
        with torch.cuda.stream(side):
            g.capture_begin()
            body(twin, opts[1], 1, images)
            g.capture_end()
        assert images.hits > h
        md.captured_metadata()
        cur = torch.cuda.current_stream()
        cur.wait_event(ev)
        g.replay()
        torch.cuda.synchronize()
        _same(model, twin, opts)
    finally:
        scn.weight_images.disable()


def test_replaced_storage_drops_its_images():
    """A parameter whose storage is replaced after its images were recorded (`p.data = ...`) loses them at the next
    prepare(): no split reads the old buffer, the convolutions split the new weights, and the results equal a
    model that never had images."""
    model, xs, ys = _model()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    images = scn.weight_images.enable(model, optimizer=opt)
    try:
        for k in range(2):
            images.prepare()
            opt.zero_grad(set_to_none=True)
            logits, _ = model((xs[k % 2], None), istrain=True)
            F.multilabel_soft_margin_loss(logits, ys[k % 2]).backward()
            opt.step()
        n0 = len(images.entries)
        conv = next(m for m in model.modules() if isinstance(m, scn.SubmanifoldConvolution) and m.nIn == 32)
        old_ptr = conv.weight.data_ptr()
        conv.weight.data = conv.weight.data.clone() * 1.5   # new storage; the old one is freed
        assert conv.weight.data_ptr() != old_ptr
        images.prepare()
        assert len(images.entries) < n0
        assert all(e[0].wt != old_ptr for e in images.entries.values())
        twin = copy.deepcopy(model)
        scn.weight_images._ACTIVE = images
        with torch.no_grad():
            a, _ = model((xs[0], None), istrain=True)
        scn.weight_images._ACTIVE = None
        with torch.no_grad():
            b, _ = twin((xs[0], None), istrain=True)
        assert torch.equal(a, b)
    finally:
        scn.weight_images.disable()
