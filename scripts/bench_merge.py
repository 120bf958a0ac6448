"""Device batch assembly vs the numpy collate (trainMerge restatement) on the
headline batch (8 rooms, scale 50): wall time per batch."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
from wsss3d.merge import DeviceScenes, train_merge_gpu
from wsss3d.synthetic import make_room, train_merge
scenes = [make_room(i) for i in range(8)]
t0 = time.perf_counter()
for s in range(3):
    ref = train_merge(scenes, 50, seed=s)
cpu = (time.perf_counter() - t0) / 3
sc = DeviceScenes(scenes)
for s in range(3):
    train_merge_gpu(sc, 50, seed=s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in range(10):
    b = train_merge_gpu(sc, 50, seed=s)
torch.cuda.synchronize()
gpu = (time.perf_counter() - t0) / 10
print(f"points {sc.start[-1]}  numpy trainMerge {cpu * 1e3:.1f} ms/batch (1 core)  device {gpu * 1e3:.2f} ms/batch "
      f"(incl. the batch_offsets host read)  x{cpu / gpu:.0f}")
