"""Probe: how much of the headline step is launch gaps?  Captures one whole training step (forward on
prefetched metadata, loss, backward, fused Adam) of the bench's C3 workload into a HIP graph and replays it,
against the same step run eagerly.  Upper bound only (the replay reuses one batch's capture); the product
path captures every step afresh (bench.py --graph).  Usage: python scripts/graph_probe.py (env STEPS)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import __graft_entry__ as g_  # noqa: E402

g_.add_path()
import torch  # noqa: E402

import sparseconvnet as scn  # noqa: E402
from sparseconvnet import _lib  # noqa: E402
from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY  # noqa: E402
from wsss3d.synthetic import make_batch  # noqa: E402

_lib.load()
dev = torch.device("cuda:0")
b = make_batch(8, 50, seed=0)
x = EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
             batch_offsets=b["batch_offsets"])
y = torch.from_numpy(b["scene_labels"]).to(dev)
torch.manual_seed(0)
pc = EasyDict(name="SparseConvUNet", m=32, dimension=3, full_scale=4096, block_reps=2, residual_blocks=True)
cls, _ = MODEL_REGISTRY.get("MultiLabel")
model = cls(pc).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
loss_fn, _ = LOSS_REGISTRY.get("Classification")
steps = int(os.environ.get("STEPS", "20"))


def step():
    opt.zero_grad(set_to_none=True)
    logits, _ = model((x, None), istrain=True)
    loss = loss_fn(logits, y)
    loss.backward()
    opt.step()
    return loss


def eager(n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        scn.prefetch_metadata(model, x.coords, wait_for_producer=False)
        step()
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t) / n


for _ in range(3):
    scn.prefetch_metadata(model, x.coords, wait_for_producer=False)
    step()
print(f"eager (prefetch each step): {eager(steps):.2f} ms/step", flush=True)

scn.prefetch_metadata(model, x.coords, wait_for_producer=False)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
t0 = time.perf_counter()
with torch.cuda.stream(s):
    g.capture_begin()
    step()
    g.capture_end()
t1 = time.perf_counter()
from sparseconvnet import metadata as scn_meta  # noqa: E402
keep = scn_meta.captured_metadata()
assert keep, "the captured forward did not consume the prefetched metadata"

torch.cuda.synchronize()
print(f"capture {1e3 * (t1 - t0):.1f} ms host", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(steps):
    g.replay()
torch.cuda.synchronize()
print(f"graph replay: {1e3 * (time.perf_counter() - t) / steps:.2f} ms/step", flush=True)

# can a kernel be timed inside a captured graph?  event record nodes around one launch, elapsed time after replay
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
g2 = torch.cuda.CUDAGraph()
a = torch.randn(4096, 4096, device=dev)
with torch.cuda.stream(s):
    g2.capture_begin()
    e0.record()
    bb = a @ a
    e1.record()
    g2.capture_end()
g2.replay()
torch.cuda.synchronize()
try:
    print(f"event nodes in a graph: elapsed {e0.elapsed_time(e1):.3f} ms", flush=True)
except Exception as ex:  # noqa: BLE001
    print(f"event nodes in a graph: no timing ({ex})", flush=True)

# fresh graph per step (what bench.py --graph does): host cost of the first replay and device time per replay,
# with and without uploading the executable graph ahead (hipGraphUpload on a side stream)
import ctypes  # noqa: E402
hip = ctypes.CDLL("libamdhip64.so")
hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for upload in (False, True):
    res = []
    for k in range(6):
        scn.prefetch_metadata(model, x.coords, wait_for_producer=False)
        ev = scn_meta.prefetch_event(dev)
        torch.cuda.synchronize()
        gk = torch.cuda.CUDAGraph()
        tc = time.perf_counter()
        with torch.cuda.stream(s):
            gk.capture_begin()
            step()
            gk.capture_end()
        tc = time.perf_counter() - tc
        keepk = scn_meta.captured_metadata()
        tu = time.perf_counter()
        if upload:
            rc = hip.hipGraphUpload(ctypes.c_void_p(gk.raw_cuda_graph_exec()), ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc
            s.synchronize()
        tu = time.perf_counter() - tu
        cur = torch.cuda.current_stream()
        cur.wait_event(ev)
        a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a0.record()
        th = time.perf_counter()
        gk.replay()
        th = time.perf_counter() - th
        a1.record()
        torch.cuda.synchronize()
        res.append((1e3 * tc, 1e3 * tu, 1e3 * th, a0.elapsed_time(a1)))
    print(f"fresh graphs, upload={upload}: capture / upload / replay-call host ms, device ms:",
          [tuple(round(v, 1) for v in r) for r in res], flush=True)
