"""Data parallelism for the encoder step: one process per GPU, scenes sharded
across ranks, gradients averaged by DDP over RCCL (xGMI).

The reference trains on one GPU and has no distributed code (SURVEY.md §0.2,
§8(e)); `options: [distributed]` in
`config/3DUNetWithText_scannet_subcloud_uppool_4gpu.yaml:28-29` is never read.
Scenes are independent, every sparse op is local to a rank's batch, and the
only exchange is the gradient all-reduce, so this is plain DDP:

* `init_from_env()` reads torchrun's RANK / LOCAL_RANK / WORLD_SIZE and
  initialises the process group ("nccl" = RCCL on ROCm when a GPU is used,
  "gloo" otherwise);
* `balanced_shards()` assigns scenes to ranks by point count (longest
  processing time first) so per-rank step times stay close -- the step is
  bound by the slowest rank;
* `wrap()` builds DDP with local BatchNorm statistics (broadcast_buffers=False,
  as in a single-GPU reference run at the per-rank batch size; no SyncBN) and
  gradient buckets sized for ring all-reduce over xGMI;
* `GradSync` is the same exchange for steps captured into HIP graphs (no DDP
  hooks inside a capture): the gradients are views of one flat buffer that the
  captured backward accumulates into in place, and one all-reduce over it runs
  eagerly between the graph's replay and the optimizer step.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(device_type: str = "cuda", backend: str | None = None, device_index: int | None = None):
    """Returns (rank, world, local_rank, device).  backend: "nccl" (RCCL, the
    default on GPUs) or "gloo" (the default on CPU; also lets several ranks
    share one GPU in tests, which RCCL refuses).  device_index overrides
    LOCAL_RANK as the GPU this rank uses."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type == "cuda":
        idx = local if device_index is None else int(device_index)
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = backend or ("nccl" if device_type == "cuda" else "gloo")
        # RCCL's communicator is created lazily, at the first collective (no device_id): bound eagerly, it
        # made every later device-to-host read wait for ALL queued work on the device, not just its own
        # stream -- the metadata prefetch's count reads then stalled behind the running step (82.8 vs
        # 60.1 ms/step with a one-rank group, profiles/r02/bench_dp_selftest_r02.log)
        dist.init_process_group(backend)
    return rank, world, local, device


def balanced_shards(sizes, world: int):
    """Split scene indices into `world` shards of equal count (the remainder
    is dropped, like the reference's drop_last loader, dataset/data.py:239-247)
    balancing the total point count: scenes are taken in decreasing size and
    each goes to the lightest shard that still has room."""
    n = len(sizes) // world * world
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))[:n]
    per = n // world
    shards = [[] for _ in range(world)]
    load = [0] * world
    for i in order:
        r = min((r for r in range(world) if len(shards[r]) < per), key=lambda r: (load[r], r))
        shards[r].append(i)
        load[r] += sizes[i]
    return [sorted(s) for s in shards]


def wrap(model, device, bucket_cap_mb: int = 64):
    """DDP with local BN statistics.  64 MB buckets: the headline UNet's 120 MB
    of fp32 gradients go out in two ring all-reduces, each large enough to
    run every xGMI link at full rate, overlapped with the rest of backward."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return model
    ids = [device.index] if device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, broadcast_buffers=False,
                                                     bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)


class GradSync:
    """Data-parallel gradient averaging for graph-captured steps.

    DDP all-reduces from autograd hooks while backward runs; a HIP graph that
    captures the backward would capture those collectives as well.  Here the
    step's forward + backward is the graph and the exchange stays outside it:
    the parameters start equal on every rank (broadcast from rank 0, as DDP's
    constructor does), every gradient is a view of one flat fp32 buffer (so
    the captured backward writes it in place and the step zeroes it with
    ``zero_grad(set_to_none=False)``), and `average()` issues ONE all-reduce
    over the whole buffer (120 MB for the headline UNet: one large RCCL ring
    all-reduce over xGMI, ~1 ms) followed by the 1/world scaling -- the same
    mean DDP computes.  BN buffers stay local (as `wrap`, broadcast_buffers=False)."""

    def __init__(self, model, device):
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, 0)
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError("GradSync: fp32 parameters only")
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            off += p.numel()

    def check_views(self):
        """The gradients must still be the flat buffer's views (a zero_grad(set_to_none=True) or a
        non-accumulating backward would have replaced them)."""
        off = 0
        for p in self.params:
            g = p.grad
            if g is None or g.data_ptr() != self.flat[off:off + p.numel()].data_ptr():
                raise RuntimeError("GradSync: a gradient is no longer a view of the flat buffer")
            off += p.numel()

    def average(self):
        if dist.is_initialized():
            dist.all_reduce(self.flat)
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)


def max_over_ranks(x: float) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64,
                     device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(x: float) -> list:
    """[x of rank 0, x of rank 1, ...] (a one-element list without a process group)."""
    if not dist.is_initialized():
        return [x]
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(v.item()) for v in out]


def sum_over_ranks(x: float) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64,
                     device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
