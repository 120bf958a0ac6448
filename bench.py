"""Headline benchmark: active-voxels/sec of one SparseConvUNet training step.

Workload (BASELINE.json configs[2], the metric's config): SparseConvUNet m=32,
block_reps=2, residual blocks, scale 50 (2 cm voxels), 8 synthetic
ScanNet-shaped scenes per GPU, MultiLabel head + multilabel soft-margin loss.
A step = zero_grad -> forward (metadata built on the device from raw coords)
-> loss -> backward -> Adam step, on batches already resident in HBM.
value = sum over ranks of level-0 active voxels per step x steps / max-over-
ranks wall time.  N>1: one process per GPU, each rank its own scenes (weak
scaling), DDP gradient all-reduce over RCCL.  `python bench.py --gpus N`
without torchrun's environment starts the N ranks itself (a torch.distributed.run
child, launched before this process touches the GPU) and passes rank 0's line
through.  --preset c2/c3/c4/c5 selects BASELINE.json configs[1..4] (c4 =
the headline network at 5 scenes per GPU).

Also reported: roofline of the dominant kernel family (msp_conv_tile /
msp_conv_nbr: bf16 MFMA on exact three-piece splits -- six bf16 products per
fp32 multiply-add -- so the peak is 2500/6 TF/s fp32-equivalent; a call on the
f32-MFMA forms would be priced at 157.3 and the peak reported is the
FLOP-weighted mix) and of every other recorded family (weight gradients,
one-contribution convolutions, NetworkInNetwork, BatchNorm), each call timed
live with HIP events on its launch stream during the timed steps; the
step-level roofline of SURVEY.md §8(d) (t_roof = max(B_alg / 8 TB/s,
F_alg / peak), F_alg = 6 x the forward multiply-add counter); and the CPU
oracle path (fp32, all host cores available to the process) on a bounded
sample on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "3d-weakly-supervised-semantic-segmentation_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table (f32 MFMA = f32 vector peak)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # same table, dense
# split-bf16 ("x6") convolutions: six bf16 MFMA products per fp32 multiply-add
X6_PEAK_TFLOPS = BF16_MFMA_PEAK_TFLOPS / 6.0
HBM_PEAK_GBS = 8000.0

# recorded kinds (sparseconvnet/ops.py _record) -> family
CONV_KINDS = ("subm_fwd", "conv_fwd", "subm_bwd_data", "deconv_bwd_data")
FAMILIES = {"wgrad": "wgrad", "nin_wgrad": "wgrad", "wgrad_strided": "wgrad", "wgrad_deconv": "wgrad",
            "conv_bwd_data": "pairs", "deconv_fwd": "pairs",
            "nin_fwd": "nin", "nin_bwd_data": "nin", "bn_fwd": "bn", "bn_bwd": "bn", "bn_join": "bn"}


_HIP_RT = None  # ctypes handle of the HIP runtime (bench.py --graph-upload)

def family(kind):
    base = kind.split("/")[0]
    return "conv" if base in CONV_KINDS else FAMILIES.get(base, base)


def kind_peak(kind):
    return X6_PEAK_TFLOPS if "/x6" in kind else FP32_MFMA_PEAK_TFLOPS


PRESETS = {  # BASELINE.json configs[1..4]
    "c2": dict(workload="unet", m=16, reps=1, residual=0, scale=50, batch=4),
    "c3": dict(workload="unet", m=32, reps=2, residual=1, scale=50, batch=8),
    "c4": dict(workload="unet", m=32, reps=2, residual=1, scale=50, batch=5),
    "c5": dict(workload="contrastive", m=32, reps=1, residual=0, scale=20, batch=8),
}


class KernelRecorder:
    """Brackets every recorded library call (sparseconvnet/ops.py _record: the conv family, weight
    gradients, one-contribution convolutions, NetworkInNetwork, BatchNorm) with torch.cuda.Events on the
    current stream -- the stream the kernels are launched on -- and accumulates each call's algorithmic
    FLOPs and compulsory bytes.  mode "conv" records the conv family only."""

    def __init__(self, mode="all", pool=8192):
        self.events = []
        self.active = False
        self.mode = mode
        # events created up front and reused: creating two per call inside the timed steps cost ~3 ms of host
        # time per step
        self.pool = [torch.cuda.Event(enable_timing=True) for _ in range(pool if mode != "none" else 0)]
        self.used = 0

    def run(self, kind, flops, fn, nbytes=0):
        if not self.active or (self.mode == "conv" and family(kind) != "conv"):
            return fn()
        if self.used + 2 <= len(self.pool):
            s, e = self.pool[self.used], self.pool[self.used + 1]
            self.used += 2
        else:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.events.append((kind, flops, nbytes, s, e))
        return r

    def summary(self):
        """family -> {achieved, peak, frac, bound, unit, ms, launches, bytes, gbs, per_kind}."""
        torch.cuda.synchronize()
        per = {}
        for kind, f, nb, s, e in self.events:
            k = per.setdefault(kind, [0, 0.0, 0.0, 0.0])
            k[0] += 1
            k[1] += f
            k[2] += nb
            k[3] += s.elapsed_time(e)
        fams = {}
        for kind, (n, f, nb, ms) in per.items():
            d = fams.setdefault(family(kind), {"launches": 0, "flops": 0.0, "bytes": 0.0, "ms": 0.0,
                                               "t_peak": 0.0, "per_kind": {}})
            d["launches"] += n
            d["flops"] += f
            d["bytes"] += nb
            d["ms"] += ms
            d["t_peak"] += f / (kind_peak(kind) * 1e12)
            sec = ms * 1e-3
            d["per_kind"][kind] = {"launches": n, "ms": ms,
                                   "tflops": f / sec / 1e12 if sec and f else 0.0,
                                   "gbs": nb / sec / 1e9 if sec else 0.0}
        out = {}
        for fam, d in fams.items():
            sec = d["ms"] * 1e-3
            gbs = d["bytes"] / sec / 1e9 if sec else 0.0
            if d["flops"] > 0:
                achieved = d["flops"] / sec / 1e12 if sec else 0.0
                peak = d["flops"] / d["t_peak"] / 1e12 if d["t_peak"] else FP32_MFMA_PEAK_TFLOPS
                bound, unit = "mfma", "TFLOP/s"
            else:
                achieved, peak, bound, unit = gbs, HBM_PEAK_GBS, "hbm", "GB/s"
            out[fam] = {"bound": bound, "achieved": achieved, "peak": peak, "unit": unit,
                        "frac": achieved / peak if peak else 0.0, "ms": d["ms"], "launches": d["launches"],
                        "bytes": d["bytes"], "gbs": gbs, "per_kind": d["per_kind"]}
        return out


def pmc_traffic():
    """HBM bytes per conv-family call measured with rocprofv3 PMC counters on this workload
    (scripts/pmc_traffic.sh; committed under profiles/, newest round first), or None."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")
        if os.path.isfile(path):
            break
    else:
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_call"), os.path.relpath(path, ROOT)


def level_stats(meta):
    out = []
    for size in sorted(meta.levels, reverse=True):
        lvl = meta.levels[size]
        r = lvl.subm.get(3)
        out.append({"size": size, "V": lvl.n, "R": (r.n_rules if r else None)})
    return out


def host_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota if one is set (on
    the GPU box os.cpu_count() reports the whole machine while the job gets a share of it)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    cores = max(1, min(n, int(math.ceil(quota))) if quota else n)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return cores, {"affinity_cpus": n, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
                   "cpu_model": model}


def cpu_baseline(args, batch, iters=3):
    """CPU oracle (fp32, SCN-CPU-structured gather -> MKL mm -> scatter-add, torch threads = every core
    available to the process) on a bounded sample: the first scene of the batch, one warm-up then the
    median of `iters` fwd+bwd steps (each step rebuilds the voxelisation and rulebooks, as SCN's CPU
    path does per forward)."""
    from oracle.encoders import OracleEncoder

    cores, info = host_cores()
    threads = int(os.environ.get("BENCH_CPU_THREADS", cores))
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    off = batch["batch_offsets"]
    n0 = off[1]
    coords = torch.from_numpy(batch["coords"][:n0])
    feats = torch.from_numpy(batch["feats"][:n0])
    torch.manual_seed(0)
    ref = OracleEncoder("SparseConvUNet", m=args.m, full_scale=4096, block_reps=args.reps,
                        residual_blocks=bool(args.residual))
    lin = torch.nn.Linear(args.m, 20)
    y = torch.from_numpy(batch["scene_labels"][:1])
    x = dict(coords=coords, feature=feats, batch_offsets=[0, n0])
    times = []
    for it in range(iters + 1):
        ref.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        feats_out = ref(x, istrain=True)
        loss = torch.nn.functional.multilabel_soft_margin_loss(lin(feats_out), y)
        loss.backward()
        dt = time.perf_counter() - t0
        if it:
            times.append(dt)
    torch.set_num_threads(prev)
    med = statistics.median(times)
    V0 = len(np.unique(batch["coords"][:n0], axis=0))
    return {"value": V0 / med, "unit": "active-voxels/s", "cores": threads, "kind": "port",
            "cpu_model": info["cpu_model"], "host": info,
            "sample": f"1 scene of the workload ({n0} points, {V0} L0 voxels), fwd+bwd, fp32, "
                      f"oracle/scn_oracle.py on {threads} torch threads: 1 warm-up + median of {iters} "
                      f"({', '.join(f'{t:.2f}' for t in times)} s)"}


def balanced_batch(args, rank, world, k):
    """Batch k of this rank under LPT assignment: the same pool of world x batch procedural rooms on every rank
    (seeded by k), sharded by point count with wsss3d.dp.balanced_shards, then this rank's rooms through the
    trainMerge transform (dataset/data.py:135-238) as make_batch does."""
    from wsss3d import dp
    from wsss3d.synthetic import make_room, train_merge
    pool = [make_room((100 + k) * 1000 + i) for i in range(world * args.batch)]
    sizes = [len(room[0]) for room in pool]
    shard = dp.balanced_shards(sizes, world)[rank]
    return train_merge([pool[i] for i in shard], args.scale, 4096, 1000 * rank + k)


def launch_ranks(n):
    """Start n ranks (torch.distributed.run child, one process per GPU) before this process touches the
    GPU; rank 0 prints the JSON line.  Returns the child's exit code."""
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--preset", choices=sorted(PRESETS), default=None,
                    help="BASELINE.json configs[1..4]: c2 UNet m16 r1 VGG b4, c3 (default) UNet m32 r2 residual b8, "
                         "c4 the same at 5 scenes per GPU, c5 MultiLabelContrastive FCNet m32 + text")
    ap.add_argument("--batch", type=int, default=None, help="scenes per GPU (default 8)")
    ap.add_argument("--scale", type=float, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--reps", type=int, default=None)
    ap.add_argument("--residual", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-iters", type=int, default=3, help="timed cpu_baseline iterations (median)")
    ap.add_argument("--record", choices=["all", "conv", "none"], default="conv",
                    help="HIP-event bracketing of the recorded calls in the timed steps (roofline): the conv "
                         "family only (default), every recorded family, or none.  Every bracketed call costs "
                         "about 2.5 us of stream time (all families: ~3 ms per step), so the other families' "
                         "rooflines come from --family-steps extra recorded steps after the timed region")
    ap.add_argument("--family-steps", type=int, default=5,
                    help="untimed steps after the timed region with every family recorded (per-family rooflines "
                         "and the step-level compulsory bytes); 0 = none")
    ap.add_argument("--foreach-adam", action="store_true", help="torch's foreach Adam instead of the fused one")
    ap.add_argument("--adam", choices=["library", "torch"], default="library",
                    help="library: the reference's Adam update in one launch over every parameter (wsss3d.optim.Adam, "
                         "msp_adam_step); torch: torch.optim.Adam (fused multi-tensor, or --foreach-adam)")
    ap.add_argument("--concurrent-wgrad", action="store_true",
                    help="every weight gradient on a side stream beside the backward-data (sparseconvnet.ops)")
    ap.add_argument("--compute-priority", type=int, choices=[0, 1], default=0,
                    help="1: run the step on a high-priority stream (the metadata prefetch keeps the default one)")
    ap.add_argument("--wgrad-side-rows", type=int, default=None,
                    help="levels below this many rows run the weight gradient beside the backward-data "
                         "(sparseconvnet.ops.WGRAD_SIDE_ROWS; 0 = never)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="build each batch's metadata inside its own forward (no side-stream input pipelining)")
    ap.add_argument("--prefetch-priority", type=int, choices=[0, 1], default=0,
                    help="1: the metadata prefetch on a high-priority stream (its small kernels and the count reads "
                         "the host waits on no longer queue behind the running step's workgroups)")
    ap.add_argument("--prefetch-lag", type=int, choices=[1, 2], default=1,
                    help="graph mode: the metadata build of batch i + 1 waits for step i - lag's graph (1: the host "
                         "runs at most one step ahead; 2: two)")
    ap.add_argument("--prefetch-thread", type=int, choices=[0, 1], default=0,
                    help="graph mode, 1: the metadata of the batch after next is built on a worker thread while the "
                         "next step is captured (two prefetched batches pending; the build waits for the step two "
                         "back); 0: prefetch, then capture, on the loop's thread")
    ap.add_argument("--prefetch-at", choices=["end", "fwd"], default="end",
                    help="when the next batch's metadata is built: after the step's optimizer call is queued (end) "
                         "or right after its forward is queued (fwd: the build's host reads overlap the forward)")
    ap.add_argument("--meta-release", choices=["done", "stream"], default="done",
                    help="graph mode: when a replayed step's metadata is freed -- done: once the step's end event has "
                         "completed (polled on the host, nothing queued on the device); stream: right after the "
                         "replay is queued, its tensors marked as used by the compute stream (the caching allocator "
                         "then records one event per freed block on that stream: ~1.1 ms of device idle per step)")
    ap.add_argument("--graph-upload", type=int, choices=[0, 1], default=0,
                    help="graph mode, 1: each captured graph is uploaded (hipGraphUpload) on the capture stream right "
                         "after its capture, while the previous step runs; the replay waits for the upload")
    ap.add_argument("--graph", type=int, choices=[0, 1], default=None,
                    help="1: capture every step afresh into a HIP graph (built after the step's metadata is "
                         "prefetched, replayed on the compute stream while the next step is prefetched and "
                         "captured; N ranks: forward + backward captured, the gradient all-reduce and Adam eager after each "
                         "replay) -- removes the per-kernel launch gaps; default 1")
    ap.add_argument("--weight-images", type=int, default=1, choices=[0, 1],
                    help="1: split every convolution's weight image of a step in one launch at its start "
                         "(sparseconvnet.weight_images); 0: each call splits its own")
    ap.add_argument("--balance", choices=["none", "lpt"], default="none",
                    help="scene assignment over ranks: none = every rank draws its own scenes (weak scaling, the "
                         "default); lpt = all ranks' scenes drawn from one pool and assigned by point count, "
                         "longest first, to the lightest rank (wsss3d.dp.balanced_shards), so the slowest rank's "
                         "step is as short as the pool allows")
    ap.add_argument("--workload", choices=["unet", "contrastive"], default=None,
                    help="unet: the headline config (BASELINE configs[2]); contrastive: configs[4] per GPU -- "
                         "MultiLabelContrastive = SparseConvFCNet m=32 r1 at scale 20 + TextTransformer "
                         "(CLIP text-tower shape: width 512, 12 layers, context 120, vocab 49408), 10 texts per "
                         "scene, Classification + TextContrastive losses")
    args = ap.parse_args()
    preset = args.preset or ("c5" if args.workload == "contrastive" else "c3")
    for k, v in PRESETS[preset].items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    from wsss3d import dp

    # BENCH_BACKEND=gloo BENCH_SHARE_DEVICE=1: rehearse N ranks on a one-GPU box (RCCL refuses two ranks on
    # one device); the measured configuration is RCCL with one GPU per rank
    rank, world, local, dev = dp.init_from_env("cuda", backend=os.environ.get("BENCH_BACKEND") or None,
                                               device_index=0 if os.environ.get("BENCH_SHARE_DEVICE") else None)
    if os.environ.get("BENCH_DP_SELFTEST") and world == 1:
        # a one-rank RCCL group: runs the N-rank graph path (eager all-reduce between per-step captures) on a
        # one-GPU box, as a rehearsal of what the driver's multi-GPU runs execute
        sock = socket.socket()
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
        sock.close()
        be = "gloo" if os.environ["BENCH_DP_SELFTEST"] == "gloo" else "nccl"
        dist.init_process_group(be, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    # N ranks on one host: each rank's torch intra-op pool bounded to its share of the CPUs the job may use (the
    # default sizes it by every core the machine reports, so N ranks oversubscribe a cgroup quota N x cores-fold;
    # BENCH_THREADS overrides)
    host_threads = None
    if world > 1:
        local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        host_threads = int(os.environ.get("BENCH_THREADS", max(1, host_cores()[0] // max(local, 1))))
        torch.set_num_threads(host_threads)
    if rank == 0 and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting the {world} ranks that run",
              file=sys.stderr)

    if args.compute_priority:
        # the step's kernels on a high-priority stream: the metadata prefetch (side stream, default priority)
        # gets the CUs the step leaves idle instead of competing for them
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=-1))

    import sparseconvnet as scn
    from sparseconvnet import _lib
    from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY
    from wsss3d.synthetic import make_batch

    _lib.load()
    from sparseconvnet import ops as scn_ops
    from sparseconvnet import metadata as scn_md
    scn_md.PREFETCH_PRIORITY = -1 if args.prefetch_priority else 0
    scn_ops.WGRAD_CONCURRENT = bool(args.concurrent_wgrad)
    if args.wgrad_side_rows is not None:
        scn_ops.WGRAD_SIDE_ROWS = args.wgrad_side_rows
    # two distinct batches per rank, alternated step to step
    if args.balance == "lpt" and world > 1:
        host_batches = [balanced_batch(args, rank, world, k) for k in range(2)]
        scene_note = ("LPT over a pool of world x scenes_per_gpu scenes per batch (wsss3d.dp.balanced_shards by "
                      "point count)")
    else:
        host_batches = [make_batch(args.batch, args.scale, seed=1000 * rank + k) for k in range(2)]
        scene_note = "independent random scenes per rank (seed 1000 rank + k)"
    contrastive = args.workload == "contrastive"
    n_text, seq_len, vocab = 10, 120, 49408
    batches = []
    for k, b in enumerate(host_batches):
        x = EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
                     batch_offsets=b["batch_offsets"])
        y = torch.from_numpy(b["scene_labels"]).to(dev)
        v0 = len(np.unique(b["coords"], axis=0))
        text = None
        if contrastive:  # every scene has texts: random ids, end-of-text = the largest id
            g = torch.Generator().manual_seed(1000 * rank + k)
            tok = torch.randint(1, vocab - 1, (args.batch, n_text, seq_len), generator=g)
            eot = torch.randint(8, seq_len, (args.batch, n_text), generator=g)
            tok.scatter_(2, eot[..., None], vocab - 1)
            tok = torch.where(torch.arange(seq_len)[None, None] > eot[..., None], torch.zeros_like(tok), tok)
            text = (tok.to(dev), torch.arange(args.batch, device=dev))
        batches.append((x, y, v0, text))

    # HIP-graph steps (--graph), metadata prefetched.  One rank: the whole step (Adam included) is the graph.
    # N ranks: forward + backward are the graph, and the gradient all-reduce (one RCCL call over a flat buffer,
    # dp.GradSync) and Adam run eagerly after its replay -- DDP's hooks would otherwise be captured
    use_graph = bool(args.graph if args.graph is not None else not contrastive) \
        and not args.no_prefetch \
        and args.prefetch_at == "end"
    graph_dp = use_graph and (world > 1 or dist.is_initialized())
    wrap = (lambda m: m) if graph_dp else (lambda m: dp.wrap(m, dev))
    torch.manual_seed(0)
    if contrastive:
        pc = EasyDict(name="SparseConvFCNet", m=args.m, dimension=3, full_scale=4096, block_reps=args.reps,
                      residual_blocks=bool(args.residual))
        tc = EasyDict(name="TextTransformer", context_length=seq_len, width=512, layers=12, vocab_size=vocab)
        cls, _ = MODEL_REGISTRY.get("MultiLabelContrastive")
        model = wrap(cls(pc, tc).to(dev))
    else:
        pc = EasyDict(name="SparseConvUNet", m=args.m, dimension=3, full_scale=4096, block_reps=args.reps,
                      residual_blocks=bool(args.residual))
        cls, _ = MODEL_REGISTRY.get("MultiLabel")
        model = wrap(cls(pc).to(dev))
    n_params = sum(p.numel() for p in model.parameters())
    # the reference's optimizer (train.py:39, Adam lr 1e-3): by default its update in one library launch over
    # every parameter (wsss3d.optim.Adam); --adam torch: torch's fused multi-tensor kernels (12 launches per step),
    # --foreach-adam: torch's default foreach form (~21)
    # N ranks over RCCL: the bucket all-reduces are captured into the step's graph, issued as each bucket's
    # gradients become final, so they run beside the rest of the backward (dp.GradSync overlap);
    # BENCH_GRAD_OVERLAP=0 restores one all-reduce over the whole buffer after each replay
    overlap = graph_dp and dist.is_initialized() and dist.get_backend() == "nccl" and \
        os.environ.get("BENCH_GRAD_OVERLAP", "1") != "0"
    gsync = dp.GradSync(model, dev, overlap=overlap) if graph_dp else None
    if args.adam == "library" and not args.foreach_adam:
        from wsss3d.optim import Adam as LibAdam
        opt = LibAdam(model.parameters(), lr=1e-3)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, **({"foreach": True} if args.foreach_adam else
                                                               {"fused": True, "capturable": use_graph}))
    # every convolution's split-bf16 weight image of a step in one launch at its start (sparseconvnet.weight_images;
    # the optimizer's steps invalidate them)
    wimg = scn.weight_images.enable(model, dev, optimizer=opt) if args.weight_images else None
    cls_loss, _ = LOSS_REGISTRY.get("Classification")
    con_loss, _ = LOSS_REGISTRY.get("TextContrastive")

    prefetch_s = []

    def prefetch(i, after=None):
        # input pipelining: the next batch's voxelisation and rulebooks on a side stream while this step's
        # kernels run (sparseconvnet.prefetch_metadata); `after`: an event the build waits for
        t = time.perf_counter()
        scn.prefetch_metadata(model, batches[(i + 1) % len(batches)][0].coords,
                              wait_for_producer=after if after is not None else False)
        prefetch_s.append(time.perf_counter() - t)

    host_t = [] if os.environ.get("BENCH_HOST_TIMING") else None  # host enqueue time per phase (diagnostic)

    def step(i):
        x, y, _, text = batches[i % len(batches)]
        h0 = time.perf_counter()
        if wimg is not None:
            wimg.prepare()
        opt.zero_grad(set_to_none=gsync is None)
        logits, meta = model((x, text), istrain=True)
        h1 = time.perf_counter()
        if not args.no_prefetch and args.prefetch_at == "fwd":
            prefetch(i)
        loss = cls_loss(logits, y)
        if contrastive:
            loss = loss + con_loss(*meta)
        if gsync is not None and gsync.overlap:
            gsync.begin()
        loss.backward()
        h2 = time.perf_counter()
        if gsync is not None:
            if gsync.overlap:
                gsync.join()
            else:
                gsync.average()
        opt.step()
        h3 = time.perf_counter()
        if not args.no_prefetch and args.prefetch_at == "end":
            prefetch(i)
        if host_t is not None:
            host_t.append((h1 - h0, h2 - h1, h3 - h2, time.perf_counter() - h3))
        return loss

    from sparseconvnet import metadata as scn_meta
    cur = torch.cuda.current_stream(dev)
    cap_stream = torch.cuda.Stream(dev) if use_graph else None
    # one memory pool for every step's graph: blocks a finished step's graph freed are reused by later captures
    # (replays are ordered on the compute stream); a private pool per graph would hand its memory back with a
    # device-synchronising free each step
    graph_pool = torch.cuda.graph_pool_handle() if use_graph else None

    capture_s = []
    capture_parts = []  # BENCH_HOST_TIMING: (capture_begin, body, capture_end) host seconds

    def body(i):  # one training step without its prefetch (what a graph captures; N ranks: up to backward)
        x, y, _, text = batches[i % len(batches)]
        if wimg is not None:
            wimg.prepare()
        opt.zero_grad(set_to_none=gsync is None)
        logits, meta = model((x, text), istrain=True)
        loss = cls_loss(logits, y)
        if contrastive:
            loss = loss + con_loss(*meta)
        if gsync is not None and gsync.overlap:
            gsync.begin()
        loss.backward()
        if gsync is None:
            opt.step()
        elif gsync.overlap:
            gsync.join()  # the exchange's graph nodes rejoin the captured stream
        return loss

    def _hip_runtime():
        # the HIP runtime torch itself loaded (by soname); only --graph-upload calls into it
        global _HIP_RT
        if _HIP_RT is None:
            _HIP_RT = ctypes.CDLL("libamdhip64.so")
            _HIP_RT.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            _HIP_RT.hipGraphUpload.restype = ctypes.c_int
        return _HIP_RT

    cprof = None
    if os.environ.get("BENCH_CPROFILE"):  # diagnostic: host profile of the captures and prefetches in the loop
        import cProfile
        cprof = cProfile.Profile()

    def capture(i):
        """Graph of step i, whose metadata is the pending prefetch; returns (graph, metadata it reads, the
        metadata's build event).  Nothing executes here: the kernels run at replay."""
        t = time.perf_counter()
        if wimg is not None:
            wimg.build()  # eagerly: images and descriptor table for what the last step added
        ev = scn_meta.prefetch_event(dev, batches[i % len(batches)][0].coords)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(cap_stream):
            c0 = time.perf_counter()
            g.capture_begin(pool=graph_pool, capture_error_mode="relaxed")
            c1 = time.perf_counter()
            try:
                body(i)
            except BaseException:
                # end the capture and discard the graph before the error propagates (an open capture makes
                # ~CUDAGraph terminate the process); sparseconvnet.graphs.capture is the same path
                scn.graphs.abort(g, gsync.abort if gsync is not None else None)
                raise
            c2 = time.perf_counter()
            g.capture_end()
            c3 = time.perf_counter()
            up = None
            if args.graph_upload:
                rc = _hip_runtime().hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                                                   ctypes.c_void_p(cap_stream.cuda_stream))
                if rc != 0:
                    raise RuntimeError(f"bench.py --graph-upload: hipGraphUpload returned {rc}")
                up = torch.cuda.Event()
                up.record(cap_stream)
        if host_t is not None:
            capture_parts.append((c1 - c0, c2 - c1, c3 - c2))
        keep = scn_meta.captured_metadata()
        if gsync is not None:
            gsync.check_views()
        if not keep:
            raise RuntimeError("bench.py --graph: the captured step did not consume its prefetched metadata")
        capture_s.append(time.perf_counter() - t)
        return g, keep, ev, up

    replay_ev = []
    build_ev = []  # BENCH_HOST_TIMING: each replay's metadata build event (when the build finished on the device)
    if host_t is not None:
        scn_meta.BUILD_EVENT_TIMING = True
        scn_meta.READ_STATS = [0.0, 0]

    def replay(entry):
        g, keep, ev, up = entry
        cur.wait_event(ev)  # the metadata build (side stream) before the graph reads it
        if up is not None:
            cur.wait_event(up)
        if args.meta_release == "stream":
            for m in keep:
                for t in m.tensors():
                    t.record_stream(cur)
        if host_t is not None:
            replay_ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
            replay_ev[-1][0].record(cur)
            build_ev.append(ev)
        g.replay()
        if gsync is not None:  # N ranks: Adam after the replayed backward (+ the exchange unless captured)
            if not gsync.overlap:
                gsync.average()
            opt.step()
        done = torch.cuda.Event(enable_timing=True)
        done.record(cur)
        if host_t is not None:
            replay_ev[-1] = (replay_ev[-1][0], done)
        return done

    for i in range(args.warmup):
        step(i)
    rec = KernelRecorder(args.record if not use_graph else "none", pool=2 * 700 * args.steps)
    _lib.set_recorder(rec if args.record != "none" and not use_graph else None)
    entry = None
    worker, fut = None, None
    if use_graph and args.prefetch_thread:
        from concurrent.futures import ThreadPoolExecutor
        scn_meta.PREFETCH_DEPTH = 2
        worker = ThreadPoolExecutor(max_workers=1)
    if use_graph:  # the first step's metadata and graph, before the timed region (as eager's last warm-up does)
        prefetch(-1)
        entry = capture(0)
        if worker is not None:  # batch 1, on the worker (finished before the timed region, like batch 0)
            worker.submit(prefetch, 0).result()
    if world > 1:
        dist.barrier()
        if graph_dp:
            dp.settle(dev)  # the barrier's work retired by the watchdog before the loop captures collectives
    torch.cuda.synchronize()
    rec.active = True
    # step boundaries on the compute stream: device time per step (median reported beside the mean)
    bounds = [torch.cuda.Event(enable_timing=True)]
    bounds[0].record(cur)
    t0 = time.perf_counter()
    loop_t = []  # graph loop host seconds per step: (replay call incl. an eager exchange, prefetch, capture)
    mem_t = []  # torch's reserved device memory after each step's capture
    last_entries = []
    held = []  # --meta-release done: (metadata, end event) of replayed steps the device may still read
    if use_graph:
        inflight, dones = [], []
        for i in range(args.steps):
            h0 = time.perf_counter()
            done = replay(entry)
            bounds.append(done)
            inflight.append((entry, done, i))
            h1 = time.perf_counter()
            if worker is None:
                # batch i + 1 on the side stream, after step i - lag's graph on the device: the build's count reads
                # pace the host (lag 1: at most one step ahead -- step i is queued while step i + 1 is captured)
                prefetch(i, dones[-args.prefetch_lag] if len(dones) >= args.prefetch_lag else None)
                dones.append(done)
            else:
                # batch i + 1 was built on the worker during the last capture; batch i + 2 goes there now, after
                # step i - 1 on the device, and is built while step i + 1 is captured here (the worker waits for
                # the device with the GIL released: metadata._host)
                if fut is not None:
                    fut.result()
                dones.append(done)
                fut = worker.submit(prefetch, i + 1, dones[-2] if len(dones) >= 2 else None) \
                    if i + 2 <= args.steps else None
            h2 = time.perf_counter()
            # the graphs are kept until the loop has drained: destroying an executable graph here synchronised
            # with the device (measured: 49 ms per step of host wait, the device idle through the next capture).
            # The metadata goes as soon as the device is done with it: --meta-release done keeps it until the
            # step's end event has completed (a host poll; the build's count reads above have waited for step
            # i - lag, so step i - 1's is normally complete by now) and frees it with no device work; stream frees
            # it now, its tensors marked as used by the compute stream, and the allocator then records an event on
            # that stream per freed block -- a few hundred markers queued between this step and the next
            if host_t is not None and i + 2 >= args.steps:
                last_entries.append(inflight[-1][0])  # BENCH_HOST_TIMING: kept whole for the replays below
            if args.meta_release == "done":
                held.append((inflight[-1][0][1], done))
                held[:] = [h for h in held if not h[1].query()]
            inflight[-1] = (inflight[-1][0][0], None, i)
            h3 = time.perf_counter()
            if cprof is not None:
                cprof.enable()
            entry = capture(i + 1) if i + 1 < args.steps else None
            if cprof is not None:
                cprof.disable()
            loop_t.append((h1 - h0, h2 - h1, time.perf_counter() - h3))
            mem_t.append(torch.cuda.memory_reserved(dev))
            if host_t is not None:
                host_t.append((h1 - h0, h2 - h1, h3 - h2, time.perf_counter() - h3))
        if host_t:
            med = [1e3 * statistics.median(c) for c in zip(*host_t[-args.steps:])]
            print(f"bench.py graph loop host ms per step (median): replay call {med[0]:.2f}  prefetch {med[1]:.2f}  "
                  f"release {med[2]:.2f}  capture {med[3]:.2f}", file=sys.stderr)
            cp = [1e3 * statistics.median(c) for c in zip(*capture_parts[-args.steps:])]
            print(f"bench.py capture host ms (median): begin {cp[0]:.2f}  body {cp[1]:.2f}  end {cp[2]:.2f}",
                  file=sys.stderr)
            print("bench.py reserved device memory after each capture, GB:",
                  [round(m / 2**30, 1) for m in mem_t], file=sys.stderr)
            print(f"bench.py metadata count reads: {scn_meta.READ_STATS[1]} reads, "
                  f"{1e3 * scn_meta.READ_STATS[0]:.1f} ms of host wait in total", file=sys.stderr)
            host_t.clear()
            torch.cuda.synchronize()
            print("bench.py graph replays, device ms:", [round(a.elapsed_time(b), 1) for a, b in replay_ev],
                  file=sys.stderr)
            print("bench.py graph replays, device idle before each, ms:",
                  [round(replay_ev[k][1].elapsed_time(replay_ev[k + 1][0]), 1) for k in range(len(replay_ev) - 1)],
                  file=sys.stderr)
            # when the next step's metadata build finished, relative to the end of the step before it (> 0: the
            # replay waited for the build)
            print("bench.py metadata build done, ms after the previous step's end:",
                  [round(replay_ev[k][1].elapsed_time(build_ev[k + 1]), 2) for k in range(len(replay_ev) - 1)],
                  file=sys.stderr)
            # the last two steps' graphs replayed back to back (their metadata kept alive; nothing queued in
            # between but the events): the idle before a replay that no host work precedes -- the same graph
            # twice, two different graphs, and a graph behind a wait on its (long completed) build event
            def b2b(seq, wait=False):
                evs = []
                for e in seq:
                    if wait:
                        cur.wait_event(e[2])
                    evs.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                    evs[-1][0].record(cur)
                    e[0].replay()
                    evs[-1][1].record(cur)
                torch.cuda.synchronize()
                return ([round(a.elapsed_time(b), 2) for a, b in evs],
                        [round(evs[k][1].elapsed_time(evs[k + 1][0]), 3) for k in range(len(evs) - 1)])
            ea, eb = last_entries[-2], last_entries[-1]
            for what, seq, wait in (("one graph", [eb, eb, eb], False), ("two graphs", [ea, eb, ea, eb], False),
                                    ("one graph after its build-event wait", [eb, eb, eb], True),
                                    ("two graphs after their build-event waits", [ea, eb, ea, eb], True)):
                ms, idle = b2b(seq, wait)
                print(f"bench.py back-to-back replays, {what}: device ms {ms} idle before each {idle}",
                      file=sys.stderr)
            # freshly captured graphs (their metadata built beforehand), each replayed twice right behind a replay
            # of an old graph of the same batch (the device busy, not idling through the capture): does a graph's
            # first replay run slower than its later ones, and does an upload (hipGraphUpload) beforehand help?
            fresh = []
            for j, upload in ((0, False), (2, True)):
                k = args.steps + 1 + j
                prefetch(k - 1)
                torch.cuda.synchronize()
                e = capture(k)
                if upload:
                    rc = _hip_runtime().hipGraphUpload(ctypes.c_void_p(e[0].raw_cuda_graph_exec()),
                                                       ctypes.c_void_p(cap_stream.cuda_stream))
                    assert rc == 0, rc
                torch.cuda.synchronize()
                fresh.append(e)
            ms, idle = b2b([eb, fresh[0], fresh[0], eb, fresh[1], fresh[1]], True)
            print(f"bench.py old graph, fresh graph twice, old graph, fresh uploaded graph twice: device ms {ms} "
                  f"idle {idle}", file=sys.stderr)
            fresh = None
            last_entries.clear()
        if fut is not None:
            fut.result()
        if worker is not None:
            worker.shutdown()
    else:
        for i in range(args.steps):
            step(i)
            bounds.append(torch.cuda.Event(enable_timing=True))
            bounds[-1].record(cur)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if cprof is not None and rank == 0:
        import io
        import pstats
        out = io.StringIO()
        pstats.Stats(cprof, stream=out).sort_stats("tottime").print_stats(35)
        print(out.getvalue(), file=sys.stderr)
    step_ms = [a.elapsed_time(b) for a, b in zip(bounds[:-1], bounds[1:])]
    rec.active = False
    held.clear()  # every step has completed
    if use_graph:
        inflight = entry = None
        _lib.set_recorder(None)
    if host_t:
        med = [1e3 * statistics.median(c) for c in zip(*host_t[-args.steps:])]
        print(f"bench.py host enqueue ms per step (median): forward {med[0]:.2f}  loss+backward {med[1]:.2f}  "
              f"optimizer {med[2]:.2f}  prefetch {med[3]:.2f}  sum {sum(med):.2f}", file=sys.stderr)
    vox = sum(batches[i % len(batches)][2] for i in range(args.steps))
    dt_max, vox_all = dp.max_over_ranks(dt), dp.sum_over_ranks(float(vox))
    med_step = dp.max_over_ranks(statistics.median(step_ms))
    rank_vox = dp.gather_floats(float(vox) / args.steps)  # level-0 voxels per step of every rank
    # every rank's graph-loop host time per step (medians): where an N-rank step's wall time goes on the host
    loop_med = [1e3 * statistics.median(c) for c in zip(*loop_t)] if loop_t else [0.0, 0.0, 0.0]
    rank_host = [dp.gather_floats(v) for v in loop_med] if world > 1 else [[v] for v in loop_med]
    _lib.set_recorder(None)
    fams = rec.summary()
    fam_steps = args.family_steps if (args.record != "all" or use_graph) else 0
    if fam_steps:
        # every family bracketed, outside the timed region (see --record)
        rec_all = KernelRecorder("all", pool=2 * 700 * fam_steps)
        _lib.set_recorder(rec_all)
        rec_all.active = True
        for i in range(fam_steps):
            step(args.steps + i)
        rec_all.active = False
        _lib.set_recorder(None)
        fams_all = rec_all.summary()
        if use_graph:  # HIP events cannot time kernels inside a graph: the conv family from the recorded steps
            fams = fams_all
    else:
        fams_all = fams
        fam_steps = args.steps

    # one untimed forward for the per-level statistics and the MAC counter
    scn.forward_pass_multiplyAdd_count = 0
    inner = getattr(model, "module", model)
    x0 = batches[0][0]
    enc = inner.pc_encoder.encoder
    with torch.no_grad():
        t_in = enc[0]([x0.coords, x0.feature])
        t_out = t_in
        for mod in list(enc)[1:-1]:
            t_out = mod(t_out)
    stats = level_stats(t_in.metadata)
    macs = scn.forward_pass_multiplyAdd_count

    if rank == 0:
        ms_step = dt_max / args.steps * 1e3
        conv = fams.get("conv")
        traffic, traffic_src = pmc_traffic()
        if contrastive:
            workload = (f"MultiLabelContrastive: SparseConvFCNet m={args.m} block_reps={args.reps} scale="
                        f"{args.scale:g} ({100 / args.scale:g} cm voxels) + TextTransformer (512 wide, 12 layers, "
                        f"{n_text} texts x {seq_len} tokens per scene), {args.batch} scenes/GPU, Classification + "
                        "TextContrastive, Adam step")
        else:
            workload = (f"SparseConvUNet m={args.m} block_reps={args.reps} residual={bool(args.residual)} "
                        f"scale={args.scale:g} ({100 / args.scale:g} cm voxels), {args.batch} scenes/GPU, "
                        "MultiLabel head, Adam step")
        res = {
            "metric": "active-voxels/sec fwd+bwd, SparseConvUNet m=32 2cm voxels" if not contrastive else
                      "active-voxels/sec fwd+bwd, MultiLabelContrastive (SparseConvFCNet m=32 + TextTransformer)",
            "value": vox_all / dt_max,
            "unit": "active-voxels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "ms_per_step_median": med_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic ScanNet-shaped procedural rooms (wsss3d/synthetic.py), trainMerge transform, "
                    "random-init weights",
            "config": {
                "workload": workload,
                "preset": preset,
                "optimizer": ("Adam lr 1e-3 (train.py:39), the update in one library launch over every parameter "
                              "(wsss3d.optim.Adam, msp_adam_step)" if args.adam == "library" and not args.foreach_adam
                              else "torch.optim.Adam lr 1e-3 (train.py:39), " +
                              ("foreach" if args.foreach_adam else "fused multi-tensor")),
                "timed_step": "zero_grad -> forward (metadata from raw device coordinates) -> loss -> backward -> "
                              "Adam step; BASELINE.md's metric excludes the optimizer step, so including it is "
                              "conservative.  ms_per_step = wall time over the timed steps / steps (max over "
                              "ranks); ms_per_step_median = median device time between consecutive step "
                              "completions on the compute stream (max over ranks)",
                "scenes_per_gpu": args.batch,
                "scene_assignment": scene_note,
                "rank_l0_voxels_per_step": {"min": min(rank_vox), "max": max(rank_vox),
                                            "mean": sum(rank_vox) / len(rank_vox),
                                            "max_over_mean": max(rank_vox) / (sum(rank_vox) / len(rank_vox))},
                "global_batch": args.batch * world,
                "parallelism": f"dp{world}",
                "grad_exchange": None if not dist.is_initialized() else (
                    (f"dp.GradSync: {len(gsync.buckets)} bucket all-reduces captured into each step's graph, issued "
                     "as each bucket's gradients become final (overlapped with the rest of backward), then Adam"
                     if gsync.overlap else
                     "dp.GradSync: one all-reduce over a flat gradient buffer after each graph replay, then Adam")
                    if graph_dp else "DDP, 64 MB buckets overlapped with backward"),
                "comm_backend": dist.get_backend() if dist.is_initialized() else None,
                "host_threads_per_rank": host_threads if host_threads is not None else torch.get_num_threads(),
                "device_memory_gb": {"max_allocated": torch.cuda.max_memory_allocated(dev) / 2**30,
                                     "reserved_first_step": mem_t[0] / 2**30 if mem_t else None,
                                     "reserved_last_step": mem_t[-1] / 2**30 if mem_t else None,
                                     "note": "rank 0; torch caching allocator, graph pools included"},
                "rank_host_ms_per_step": {"replay_call_incl_eager_exchange": rank_host[0],
                                          "prefetch": rank_host[1], "capture": rank_host[2],
                                          "note": "graph loop, median per rank (rank order)"} if loop_t else None,
                "input_pipeline": "none" if args.no_prefetch else
                "next batch's metadata (voxelisation + rulebooks) built on a side stream during each step "
                f"(after its {'optimizer' if args.prefetch_at == 'end' else 'forward'} call is queued; host "
                f"time {1e3 * statistics.median(prefetch_s) if prefetch_s else 0:.1f} ms median)",
                "launch": (f"every step captured afresh into a HIP graph after its metadata is prefetched and replayed "
                           f"on the compute stream (capture host time {1e3 * statistics.median(capture_s):.1f} ms "
                           "median, overlapped with the previous step's replay)") if use_graph and capture_s else
                "eager kernel launches",
                "weight_images": (f"{len(wimg.entries)} split-bf16 weight images of the convolutions prepared in one "
                                  "launch at the start of each step (sparseconvnet.weight_images)") if wimg else
                "each convolution call splits its own weight image",
                "active_voxels_per_step_rank0": batches[0][2],
                "levels": stats,
                "fwd_multiply_adds": macs,
                "parameters": n_params,
            },
        }
        if conv is not None:
            res["roofline"] = {
                "kernel": "msp_conv_local / msp_conv_tile / msp_conv_nbr (submanifold fwd/bwd-data, strided conv fwd, "
                          "deconv bwd-data)",
                "bound": "mfma",
                "achieved": conv["achieved"],
                "peak": conv["peak"],
                "peak_note": f"mix of f32 MFMA ({FP32_MFMA_PEAK_TFLOPS} TF/s) and split-bf16 MFMA "
                             f"({BF16_MFMA_PEAK_TFLOPS:g}/6 = {X6_PEAK_TFLOPS:.1f} TF/s fp32-equivalent) weighted by "
                             "each path's FLOPs",
                "unit": "TFLOP/s",
                "frac": conv["frac"],
                "traffic": traffic,
                "traffic_unit": "HBM bytes per conv-family call (PMC 2*FETCH_SIZE + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "alg_bytes_per_call": conv["bytes"] / max(conv["launches"], 1),
                "alg_bytes_gbs": conv["gbs"],
                "launches": conv["launches"],
                "avg_launch_us": conv["ms"] / max(conv["launches"], 1) * 1e3,
                "per_kind": conv["per_kind"],
                "source": (f"{fam_steps} eagerly launched steps right after the timed region, each conv call "
                           "bracketed with HIP events on its launch stream (the timed steps run as HIP graphs, "
                           "whose kernels events cannot time; same kernels and shapes)") if use_graph else
                          "the timed steps, each conv call bracketed with HIP events on its launch stream",
            }
            res["roofline_families"] = {
                f: {k: v for k, v in d.items() if k != "per_kind" and k != "bytes"} | {"per_kind": d["per_kind"]}
                for f, d in fams_all.items()}
            res["roofline_families"]["source"] = (
                f"{fam_steps} recorded steps after the timed region (every family bracketed with HIP events)"
                if fams_all is not fams else "the timed steps")
            # step level: F_alg = 6 x forward MACs (fwd, bwd-data, bwd-weight), B_alg = the
            # compulsory bytes of every recorded call + the Adam step (param, grad, 2 moments read; 3 written)
            f_alg = 6.0 * macs
            b_rec = sum(d["bytes"] for d in fams_all.values()) / fam_steps
            b_alg = b_rec + 28.0 * n_params
            t_hbm = b_alg / (HBM_PEAK_GBS * 1e9) * 1e3
            t32 = f_alg / (FP32_MFMA_PEAK_TFLOPS * 1e12) * 1e3
            tx6 = f_alg / (X6_PEAK_TFLOPS * 1e12) * 1e3
            res["step_roofline"] = {
                "F_alg_tflop": f_alg / 1e12, "B_alg_gb": b_alg / 1e9,
                "t_roof_ms_fp32_peak": max(t_hbm, t32), "frac_fp32_peak": max(t_hbm, t32) / ms_step,
                "t_roof_ms_x6_peak": max(t_hbm, tx6), "frac_x6_peak": max(t_hbm, tx6) / ms_step,
                "hbm_frac": t_hbm / ms_step,
                "recorded_ms_per_step": sum(d["ms"] for d in fams_all.values()) / fam_steps,
                "note": "t_roof = max(B_alg / 8 TB/s, F_alg / peak); fp32 peak = 157.3 TF/s (f32 MFMA, the "
                        "arithmetic's native rate), x6 peak = 2500/6 TF/s (the split-bf16 path the convolutions "
                        "take); frac = t_roof / measured ms_per_step",
            }
        if world == 1 and not args.no_cpu and not contrastive:
            res["cpu_baseline"] = cpu_baseline(args, host_batches[0], args.cpu_iters)
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
