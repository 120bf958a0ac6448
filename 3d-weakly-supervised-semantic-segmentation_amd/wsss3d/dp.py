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

import threading
import time

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
    parameters start equal on every rank (broadcast from rank 0, as DDP's
    constructor does) and every gradient is a view of one flat fp32 buffer (so
    the captured backward writes it in place and the step zeroes it with
    ``zero_grad(set_to_none=False)``).  The buffer is laid out in reverse
    parameter order -- the order backward finalises gradients -- and cut into
    buckets of about `bucket_mb`.  Two ways to exchange it:

    * ``average()`` after the replay: ONE all-reduce over the whole buffer
      (120 MB for the headline UNet) and the 1/world scaling, eagerly.
    * overlapped (``overlap=True``, RCCL): post-accumulate-grad hooks count
      each bucket's gradients; once a bucket's last gradient is final, and
      every earlier bucket has gone out (the same order on every rank), its
      all-reduce and scaling are issued on a side stream ordered after the
      work queued so far -- inside a graph capture they are captured as graph
      nodes that run beside the rest of the backward.  ``join()`` (called at
      the end of the captured body) issues any bucket still pending and makes
      the compute stream wait for the side stream, so the optimizer after the
      replay sees the averaged gradients.

    The mean is DDP's either way (BN buffers stay local, as `wrap`,
    broadcast_buffers=False)."""

    def __init__(self, model, device, overlap: bool = False, bucket_mb: float = 32.0):
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.params = [p for p in model.parameters() if p.requires_grad]
        if self.world > 1:
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, 0)
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=device, dtype=torch.float32)
        # reverse parameter order: the buckets backward completes first come first
        order = list(reversed(self.params))
        self.buckets, self._bucket_of = [], {}
        cap = max(1, int(bucket_mb * 2 ** 20 / 4))
        off, b0, n_in = 0, 0, 0
        for p in order:
            if p.dtype != torch.float32:
                raise TypeError("GradSync: fp32 parameters only")
            p.grad = self.flat[off:off + p.numel()].view_as(p)
            self._bucket_of[p] = len(self.buckets)
            off += p.numel()
            n_in += 1
            if off - b0 >= cap:
                self.buckets.append((b0, off, n_in))
                b0, n_in = off, 0
        if n_in:
            self.buckets.append((b0, off, n_in))
        self.overlap = bool(overlap) and self.world >= 1 and dist.is_initialized()
        self._side = torch.cuda.Stream(device) if (self.overlap and device.type == "cuda") else None
        self._pending = None
        self._next = 0
        self._hooks = []
        if self.overlap and self._side is not None:
            # the process group's communicator exists before any step is captured: created lazily by a first
            # collective inside a capture, its set-up events were recorded on the capturing stream and the
            # watchdog thread's query of them failed (hipErrorCapturedEvent) on a one-rank RCCL group, where no
            # broadcast above ran first
            warm = torch.zeros(1, device=device, dtype=torch.float32)
            dist.all_reduce(warm)
            settle(device)
        if self.overlap:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def check_views(self):
        """The gradients must still be the flat buffer's views (a zero_grad(set_to_none=True) or a
        non-accumulating backward would have replaced them)."""
        off = 0
        for p in reversed(self.params):
            g = p.grad
            if g is None or g.data_ptr() != self.flat[off:off + p.numel()].data_ptr():
                raise RuntimeError("GradSync: a gradient is no longer a view of the flat buffer")
            off += p.numel()

    # ---------------------------------------------------------------- overlapped exchange
    def begin(self):
        """Start of a step's backward (overlap mode): every bucket waits for all of its gradients again."""
        self._pending = [n for (_, _, n) in self.buckets]
        self._next = 0

    def _issue(self, b):
        b0, b1, _ = self.buckets[b]
        view = self.flat[b0:b1]
        if self._side is None:  # CPU (gloo): in place, in order
            dist.all_reduce(view)
            if self.world > 1:
                view.mul_(1.0 / self.world)
            return
        cur = torch.cuda.current_stream(self.flat.device)
        self._side.wait_stream(cur)  # the bucket's gradients (and everything queued before) are final
        with torch.cuda.stream(self._side):
            dist.all_reduce(view)
            if self.world > 1:
                view.mul_(1.0 / self.world)

    def _on_grad(self, p):
        if self._pending is None:
            return
        b = self._bucket_of[p]
        self._pending[b] -= 1
        # buckets go out strictly in index order (every rank issues the same collectives in the same order)
        while self._next < len(self.buckets) and self._pending[self._next] <= 0:
            self._issue(self._next)
            self._next += 1

    def join(self):
        """End of the step's backward (overlap mode): issue what is still pending, in order, and order the
        current stream after the exchange."""
        if self._pending is None:
            return
        while self._next < len(self.buckets):
            self._issue(self._next)
            self._next += 1
        if self._side is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)
        self._pending = None

    def abort(self):
        """A capture of the step failed inside backward (sparseconvnet.graphs.capture's on_abort): the exchange
        stream rejoins the capturing stream (a stream that joined a capture and did not rejoin it keeps the
        capture from ending) and the bucket counts are dropped; the next step's begin() starts afresh."""
        if self._pending is not None and self._side is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)
        self._pending = None
        self._next = 0

    def average(self):
        if dist.is_initialized():
            dist.all_reduce(self.flat)
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)


def settle(device=None):
    """Call after the last eager collective and before a graph capture that issues collectives.

    Mechanism of the abort this removes (round 3, intermittent in the one-rank RCCL bench test): every eager
    collective's Work sits in ProcessGroupNCCL's watchdog list until the watchdog thread, on one of its passes
    (one per ~100 ms), queries the Work's end event and sees it complete.  That event was recorded on the
    communicator's stream.  A collective captured into a HIP graph makes the same stream join the capture
    (it waits on the capturing stream), and a watchdog query of an event of a stream that is capturing returns
    hipErrorCapturedEvent -- which the watchdog treats as fatal and terminates the process.  So the race is
    between the watchdog's retirement of the LAST eager collective (the communicator warm-up, the barrier) and
    the first capture.

    The fix is structural: wait until the watchdog list is empty.  ProcessGroupNCCL::waitForPendingWorks
    (`ProcessGroup._wait_for_pending_works`) returns once the watchdog has retired every enqueued Work -- it
    checks the list under the same mutex the watchdog holds while it queries events, so when it returns no
    query is in flight and none can start for Works issued before.  Captured collectives are never enqueued
    to the watchdog (ProcessGroupNCCL skips the watchdog while the stream is capturing), so after this call
    nothing the watchdog polls can meet a capture.  The device synchronisation first makes the eager
    collectives complete, so the wait is one or two watchdog passes."""
    if not (dist.is_initialized() and dist.get_backend() == "nccl"):
        return
    torch.cuda.synchronize(device)
    pg = dist.distributed_c10d._get_default_group()
    wait = getattr(pg, "_wait_for_pending_works", None)
    if wait is None:  # a torch build without the binding: wait out a few watchdog passes (the round-3 form)
        time.sleep(SETTLE_FALLBACK_S)
        return
    # bounded: the binding polls with no timeout of its own, so it runs on a helper thread with a deadline
    err = []

    def run():
        try:
            wait()
        except BaseException as e:  # noqa: BLE001 -- re-raised on the calling thread
            err.append(e)
    th = threading.Thread(target=run, name="dp-settle", daemon=True)
    th.start()
    th.join(SETTLE_TIMEOUT_S)
    if th.is_alive():
        raise RuntimeError(f"dp.settle: the process group's watchdog did not retire its pending collectives within "
                           f"{SETTLE_TIMEOUT_S:.0f} s (a collective that never completed?)")
    if err:
        raise err[0]


SETTLE_TIMEOUT_S = 120.0   # dp.settle's deadline for the watchdog to retire the eager collectives
SETTLE_FALLBACK_S = 0.35   # without _wait_for_pending_works: about three watchdog passes


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
