"""Host-side cost of one headline training step (diagnostic).

Runs the bench's C3 workload (SparseConvUNet m=32 r=2 residual, 8 scenes at 2 cm, MultiLabel head, fused
Adam, prefetched metadata) and, after warm-up, measures (1) the host enqueue time of each phase with the
device drained before the phase (so the number is host dispatch cost, not back-pressure from a full launch
queue) next to the device time of the same phase (events), and (2) a cProfile of one synchronised step,
top entries by own time.  Usage: python scripts/host_profile.py  (env STEPS, TOP; PRESET=c2 for configs[1]:
m=16, one block per level, VGG blocks, 4 scenes)."""
import cProfile
import io
import os
import pstats
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
batches = []
PRESET = os.environ.get("PRESET", "c3")
M, REPS, RES, SCENES = (16, 1, False, 4) if PRESET == "c2" else (32, 2, True, 8)
for k in range(2):
    b = make_batch(SCENES, 50, seed=k)
    x = EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
                 batch_offsets=b["batch_offsets"])
    batches.append((x, torch.from_numpy(b["scene_labels"]).to(dev)))
torch.manual_seed(0)
pc = EasyDict(name="SparseConvUNet", m=M, dimension=3, full_scale=4096, block_reps=REPS, residual_blocks=RES)
cls, _ = MODEL_REGISTRY.get("MultiLabel")
model = cls(pc).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
loss_fn, _ = LOSS_REGISTRY.get("Classification")


def phases(i, sync):
    x, y = batches[i % 2]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    host = []

    def mark(k):
        if sync:
            torch.cuda.synchronize()
        ev[k].record()
        host.append(time.perf_counter())
    mark(0)
    opt.zero_grad(set_to_none=True)
    logits, _ = model((x, None), istrain=True)
    mark(1)
    loss = loss_fn(logits, y)
    loss.backward()
    mark(2)
    opt.step()
    mark(3)
    scn.prefetch_metadata(model, batches[(i + 1) % 2][0].coords, wait_for_producer=False)
    mark(4)
    torch.cuda.synchronize()
    return [1e3 * (host[k + 1] - host[k]) for k in range(4)], [ev[k].elapsed_time(ev[k + 1]) for k in range(4)]


for i in range(4):
    phases(i, False)
steps = int(os.environ.get("STEPS", "5"))
rows = [phases(i, True) for i in range(steps)]
names = ("forward", "loss+backward", "optimizer", "prefetch")
print("phase            host enqueue ms (device drained first)   device ms (events)")
for k, n in enumerate(names):
    h = sorted(r[0][k] for r in rows)[steps // 2]
    d = sorted(r[1][k] for r in rows)[steps // 2]
    print(f"{n:16s} {h:10.2f} {d:30.2f}")

pr = cProfile.Profile()
torch.cuda.synchronize()
pr.enable()
phases(steps, True)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(int(os.environ.get("TOP", "35")))
print(s.getvalue())
