"""wsss3d.optim.Adam (the training loop's Adam, train.py:39, as one library launch per step, msp_adam_step) against
torch.optim.Adam: parameters and both moments after several steps, odd sizes (scalar path), two parameter groups,
weight decay, more tensors than one launch takes (256), a parameter without a gradient, and a captured step
replayed against eager steps."""
import pytest
import torch

import __graft_entry__ as g_

g_.add_path()
from wsss3d.optim import Adam  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(shapes, seed):
    torch.manual_seed(seed)
    return [torch.randn(*s, device=DEV) for s in shapes]


def _run(opt_cls, init, grads, groups, **kw):
    ps = [torch.nn.Parameter(t.clone()) for t in init]
    pg = [{"params": [ps[i] for i in idx], **extra} for idx, extra in groups]
    opt = opt_cls(pg, **kw)
    for step_grads in grads:
        for p, gr in zip(ps, step_grads):
            p.grad = None if gr is None else gr.clone()
        opt.step()
    torch.cuda.synchronize()
    mom = []
    for p in ps:
        st = opt.state.get(p, {})
        mom.append((st.get("exp_avg"), st.get("exp_avg_sq")))
    return [p.detach() for p in ps], mom


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_adam_matches_torch(wd):
    shapes = [(27, 64, 32), (64,), (7,), (3, 5), (1,), (33, 17), (4096, 9), (0,)]
    init = _params(shapes, 1)
    grads = [[torch.randn_like(t) for t in init] for _ in range(6)]
    groups = [(list(range(0, 4)), {}), (list(range(4, len(shapes))), {"lr": 3e-4})]
    ours, om = _run(Adam, init, grads, groups, lr=1e-3, weight_decay=wd)
    ref, rm = _run(torch.optim.Adam, init, grads, groups, lr=1e-3, weight_decay=wd, fused=True)
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=2e-7)
    for (a1, a2), (b1, b2) in zip(om, rm):
        if b1 is None:
            continue
        # moments of O(1) gradients: within an fp32 rounding of torch's (its own expression order)
        torch.testing.assert_close(a1, b1, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(a2, b2, rtol=1e-6, atol=1e-7)


def test_adam_many_tensors_and_missing_grad():
    shapes = [(int(3 + (i * 37) % 200),) for i in range(300)]  # two launches of <= 256 tensors
    init = _params(shapes, 2)
    grads = [[torch.randn_like(t) for t in init] for _ in range(3)]
    for sg in grads:
        sg[5] = None  # never gets a gradient
    ours, _ = _run(Adam, init, grads, [(list(range(300)), {})], lr=1e-3)
    ref, _ = _run(torch.optim.Adam, init, grads, [(list(range(300)), {})], lr=1e-3, fused=True)
    assert torch.equal(ours[5], init[5])
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=2e-7)


def test_adam_captured_step_replays_like_eager():
    init = _params([(128, 96), (96,), (5, 3)], 3)
    grads = [torch.randn_like(t) for t in init]
    ps_e = [torch.nn.Parameter(t.clone()) for t in init]
    ps_g = [torch.nn.Parameter(t.clone()) for t in init]
    opt_e, opt_g = Adam(ps_e, lr=1e-3), Adam(ps_g, lr=1e-3)
    for p, gr in zip(ps_e, grads):
        p.grad = gr.clone()
    for p, gr in zip(ps_g, grads):
        p.grad = gr.clone()
    opt_e.step()
    opt_g.step()  # eager first step: moments and table
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        graph.capture_begin()
        opt_g.step()
        graph.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        graph.replay()
        opt_e.step()
    torch.cuda.synchronize()
    for a, b in zip(ps_g, ps_e):
        assert torch.equal(a, b)
    assert float(opt_g.step_count) == float(opt_e.step_count) == 4.0


def test_adam_follows_moved_parameters():
    """A parameter re-homed between steps (new storage, as after load_state_dict into fresh tensors or .to()):
    the tensor table is rebuilt instead of written through a stale pointer, and the update stays torch's."""
    init = _params([(64, 48), (48,)], 4)
    grads = [[torch.randn_like(t) for t in init] for _ in range(3)]
    res = []
    for cls, kw in ((Adam, {}), (torch.optim.Adam, {"fused": True})):
        ps = [torch.nn.Parameter(t.clone()) for t in init]
        opt = cls(ps, lr=1e-3, **kw)
        for k, sg in enumerate(grads):
            if k == 1:
                ps[0].data = ps[0].data.clone()  # new storage
            for p, gr in zip(ps, sg):
                p.grad = gr.clone()
            opt.step()
        torch.cuda.synchronize()
        res.append([p.detach() for p in ps])
    for a, b in zip(*res):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=2e-7)
