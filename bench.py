"""Headline benchmark: active-voxels/sec of one SparseConvUNet training step.

Workload (BASELINE.json configs[2], the metric's config): SparseConvUNet m=32,
block_reps=2, residual blocks, scale 50 (2 cm voxels), 8 synthetic
ScanNet-shaped scenes per GPU, MultiLabel head + multilabel soft-margin loss.
A step = zero_grad -> forward (metadata built on the device from raw coords)
-> loss -> backward -> Adam step, on batches already resident in HBM.
value = sum over ranks of level-0 active voxels per step x steps / max-over-
ranks wall time.  N>1: one process per GPU (torchrun), each rank its own
scenes (weak scaling), DDP gradient all-reduce over RCCL.

Also reported: roofline of the dominant kernel (msp_conv_tile / msp_conv_nbr: bf16 MFMA on
exact three-piece splits -- six bf16 products per fp32 multiply-add -- so the
peak is 2500/6 TF/s fp32-equivalent; a call on the f32-MFMA forms would be
priced at 157.3 and the peak reported is the FLOP-weighted mix)
timed live with HIP events on its launch stream during the timed steps, and
the CPU oracle path (fp32, torch threads) on a bounded sample on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
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


def kind_peak(kind):
    return X6_PEAK_TFLOPS if kind.endswith("/x6") or kind.endswith("/x6g") else FP32_MFMA_PEAK_TFLOPS
HBM_PEAK_GBS = 8000.0


class KernelRecorder:
    """Brackets every msp_conv_tile / msp_conv_nbr launch with torch.cuda.Events on the
    current stream (the stream the kernel is launched on) and accumulates the
    algorithmic FLOPs (2 * rules * c_in * c_out) per launch."""

    def __init__(self):
        self.events = []
        self.active = False

    def run(self, kind, flops, fn, nbytes=0):
        if not self.active:
            return fn()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.events.append((kind, flops, nbytes, s, e))
        return r

    def summary(self):
        torch.cuda.synchronize()
        tot_f, tot_b, tot_ms, n = 0.0, 0.0, 0.0, 0
        per = {}
        for kind, f, nb, s, e in self.events:
            ms = s.elapsed_time(e)
            tot_f += f
            tot_b += nb
            tot_ms += ms
            n += 1
            k = per.setdefault(kind, [0, 0.0, 0.0])
            k[0] += 1
            k[1] += f
            k[2] += ms
        return tot_f, tot_b, tot_ms, n, per


def pmc_traffic():
    """HBM bytes per msp_conv_tile call measured with rocprofv3 PMC counters on
    this workload (scripts/pmc_traffic.sh; committed under profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    if not os.path.isfile(path):
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


def cpu_baseline(args, batch):
    """CPU oracle (fp32, SCN-CPU-structured gather -> mm -> scatter-add) on a
    bounded sample: the first scene of the batch, one fwd+bwd."""
    from oracle.encoders import OracleEncoder
    from wsss3d.synthetic import train_merge  # noqa: F401

    threads = int(os.environ.get("BENCH_CPU_THREADS", min(16, os.cpu_count() or 1)))
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
    t0 = time.perf_counter()
    feats_out = ref(x, istrain=True)
    loss = torch.nn.functional.multilabel_soft_margin_loss(lin(feats_out), y)
    loss.backward()
    dt = time.perf_counter() - t0
    V0 = len(np.unique(batch["coords"][:n0], axis=0))
    return {"value": V0 / dt, "unit": "active-voxels/s", "cores": threads, "kind": "port",
            "sample": f"1 scene of the workload ({n0} points, {V0} L0 voxels), 1 fwd+bwd step, fp32, "
                      f"oracle/scn_oracle.py on {threads} torch threads ({dt:.2f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="scenes per GPU")
    ap.add_argument("--scale", type=float, default=50)
    ap.add_argument("--m", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--residual", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--foreach-adam", action="store_true", help="torch's foreach Adam instead of the fused one")
    ap.add_argument("--concurrent-wgrad", action="store_true",
                    help="weight gradients on a side stream beside the backward-data (sparseconvnet.ops)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="build each batch's metadata inside its own forward (no side-stream input pipelining)")
    ap.add_argument("--workload", choices=["unet", "contrastive"], default="unet",
                    help="unet: the headline config (BASELINE configs[2]); contrastive: configs[4] per GPU -- "
                         "MultiLabelContrastive = SparseConvFCNet m=32 r1 at scale 20 + TextTransformer "
                         "(CLIP text-tower shape: width 512, 12 layers, context 120, vocab 49408), 10 texts per "
                         "scene, Classification + TextContrastive losses")
    args = ap.parse_args()
    if args.workload == "contrastive":
        if args.scale == 50:
            args.scale = 20
        args.reps, args.residual = 1, 0

    from wsss3d import dp

    rank, world, local, dev = dp.init_from_env("cuda")

    import sparseconvnet as scn
    from sparseconvnet import _lib
    from wsss3d import EasyDict, LOSS_REGISTRY, MODEL_REGISTRY
    from wsss3d.synthetic import make_batch

    _lib.load()
    from sparseconvnet import ops as scn_ops
    scn_ops.WGRAD_CONCURRENT = bool(args.concurrent_wgrad)  # set both ways (scripts/bench_ab.py reruns main)
    # two distinct batches per rank, alternated step to step
    host_batches = [make_batch(args.batch, args.scale, seed=1000 * rank + k) for k in range(2)]
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

    torch.manual_seed(0)
    if contrastive:
        pc = EasyDict(name="SparseConvFCNet", m=args.m, dimension=3, full_scale=4096, block_reps=args.reps,
                      residual_blocks=bool(args.residual))
        tc = EasyDict(name="TextTransformer", context_length=seq_len, width=512, layers=12, vocab_size=vocab)
        cls, _ = MODEL_REGISTRY.get("MultiLabelContrastive")
        model = dp.wrap(cls(pc, tc).to(dev), dev)
    else:
        pc = EasyDict(name="SparseConvUNet", m=args.m, dimension=3, full_scale=4096, block_reps=args.reps,
                      residual_blocks=bool(args.residual))
        cls, _ = MODEL_REGISTRY.get("MultiLabel")
        model = dp.wrap(cls(pc).to(dev), dev)
    # the reference's optimizer (train.py:39, Adam lr 1e-3); one fused multi-tensor kernel per step
    # (--foreach-adam: torch's default foreach form, ~21 launches per step)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, **({"foreach": True} if args.foreach_adam else {"fused": True}))
    cls_loss, _ = LOSS_REGISTRY.get("Classification")
    con_loss, _ = LOSS_REGISTRY.get("TextContrastive")

    def step(i):
        x, y, _, text = batches[i % len(batches)]
        opt.zero_grad(set_to_none=True)
        logits, meta = model((x, text), istrain=True)
        loss = cls_loss(logits, y)
        if contrastive:
            loss = loss + con_loss(*meta)
        loss.backward()
        opt.step()
        if not args.no_prefetch:
            # input pipelining: the next batch's voxelisation and rulebooks on a
            # side stream while this step's backward drains (sparseconvnet.prefetch_metadata)
            scn.prefetch_metadata(model, batches[(i + 1) % len(batches)][0].coords, wait_for_producer=False)
        return loss

    for i in range(args.warmup):
        step(i)
    rec = KernelRecorder()
    _lib.set_recorder(rec)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rec.active = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    rec.active = False
    vox = sum(batches[i % len(batches)][2] for i in range(args.steps))
    dt_max, vox_all = dp.max_over_ranks(dt), dp.sum_over_ranks(float(vox))

    flops, abytes, kms, nlaunch, per = rec.summary()
    _lib.set_recorder(None)

    # one untimed forward for the per-level statistics and the MAC counter
    scn.forward_pass_multiplyAdd_count = 0
    inner = model.module if world > 1 else model
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
        achieved = flops / (kms * 1e-3) / 1e12 if kms > 0 else 0.0
        # effective peak of the mix: the rate at which these FLOPs would run
        # if every call ran at its own path's MFMA peak
        t_peak = sum(v[1] / (kind_peak(k) * 1e12) for k, v in per.items())
        peak = flops / t_peak / 1e12 if t_peak > 0 else FP32_MFMA_PEAK_TFLOPS
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
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic ScanNet-shaped procedural rooms (wsss3d/synthetic.py), trainMerge transform, "
                    "random-init weights",
            "config": {
                "workload": workload,
                "scenes_per_gpu": args.batch,
                "global_batch": args.batch * world,
                "parallelism": f"dp{world}",
                "input_pipeline": "none" if args.no_prefetch else
                "next batch's metadata (voxelisation + rulebooks) built on a side stream during each step",
                "active_voxels_per_step_rank0": batches[0][2],
                "levels": stats,
                "fwd_multiply_adds": macs,
            },
            "roofline": {
                "kernel": "msp_conv_tile / msp_conv_nbr (submanifold fwd/bwd-data, strided conv fwd, deconv bwd-data)",
                "bound": "mfma",
                "achieved": achieved,
                "peak": peak,
                "peak_note": f"mix of f32 MFMA ({FP32_MFMA_PEAK_TFLOPS} TF/s) and split-bf16 MFMA "
                             f"({BF16_MFMA_PEAK_TFLOPS:g}/6 = {X6_PEAK_TFLOPS:.1f} TF/s fp32-equivalent) weighted by "
                             "each path's FLOPs",
                "unit": "TFLOP/s",
                "frac": achieved / peak,
                "traffic": traffic,
                "traffic_unit": "HBM bytes per msp_conv_tile / msp_conv_nbr call (PMC 2*FETCH_SIZE + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "alg_bytes_per_call": abytes / max(nlaunch, 1),
                "alg_bytes_gbs": abytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0,
                "launches": nlaunch,
                "avg_launch_us": kms / max(nlaunch, 1) * 1e3,
                "per_kind": {k: {"launches": v[0], "tflops": v[1] / (v[2] * 1e-3) / 1e12 if v[2] else 0.0,
                                 "ms": v[2]} for k, v in per.items()},
            },
        }
        if world == 1 and not args.no_cpu and not contrastive:
            res["cpu_baseline"] = cpu_baseline(args, host_batches[0])
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
