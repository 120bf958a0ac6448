"""Data parallelism around the HIP model: two ranks spawned on cuda:0 (gloo -- RCCL
refuses two ranks on one device), each running the device SparseConvUNet + MultiLabel head under
wsss3d.dp.wrap with the residual fork/join fusions on and the second step's metadata prefetched on the
side stream, as bench.py runs it.  DDP's averaged gradients must equal the mean of the ranks' local
gradients of an identical unwrapped model on the same batch, and the parameters must be identical on
both ranks after the fused Adam step."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "3d-weakly-supervised-semantic-segmentation_amd"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import torch.nn.functional as F
    import sparseconvnet as scn
    from sparseconvnet import modules
    from wsss3d import EasyDict, MODEL_REGISTRY, dp
    from wsss3d.synthetic import make_batch

    try:
        r, w, _, dev = dp.init_from_env("cuda", backend="gloo", device_index=0)
        assert modules.FUSE_RESIDUAL
        pc = EasyDict(name="SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=2,
                      residual_blocks=True)
        cls, _ = MODEL_REGISTRY.get("MultiLabel")
        torch.manual_seed(0)
        local = cls(pc).to(dev)
        torch.manual_seed(0)
        model = dp.wrap(cls(pc).to(dev), dev)
        assert isinstance(model, torch.nn.parallel.DistributedDataParallel)
        bs = [make_batch(2, 20, seed=10 * r + k) for k in range(2)]
        xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
                       batch_offsets=b["batch_offsets"]) for b in bs]
        ys = [torch.from_numpy(b["scene_labels"]).to(dev) for b in bs]

        def loss_of(net, k):
            logits, _ = net((xs[k], None), istrain=True)
            return F.multilabel_soft_margin_loss(logits, ys[k])

        # step 0 (records the rulebook plan), then the next batch's metadata on the side stream
        loss_of(model, 0).backward()
        model.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        assert scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False) is not None
        loss_of(model, 1).backward()           # consumes the prefetched metadata
        loss_of(local, 1).backward()
        ok = True
        inner = model.module
        for (k, p), q in zip(inner.named_parameters(), local.parameters()):
            g = q.grad.clone()
            dist.all_reduce(g)
            g /= w
            if not torch.allclose(p.grad, g, rtol=1e-6, atol=1e-9):
                ok = False
                print(f"rank {r}: grad {k} differs by {(p.grad - g).abs().max().item():.3e}", flush=True)
        # the two ranks' local gradients differ (different scenes), the averaged ones agree
        opt = torch.optim.Adam(inner.parameters(), lr=1e-3, fused=True)
        opt.step()
        flat = torch.cat([p.detach().flatten() for p in inner.parameters()])
        ref = flat.clone()
        dist.broadcast(ref, 0)
        ok &= torch.equal(flat, ref)
        lg = torch.cat([q.grad.flatten() for q in local.parameters()])
        other = lg.clone()
        dist.broadcast(other, 1)
        ok &= (r == 1) or not torch.equal(lg, other)
        out[rank] = bool(ok)
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        out[rank] = f"{type(e).__name__}: {e}"
        raise


def test_ddp_world2_hip_model():
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    out = manager.dict()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert dict(out) == {0: True, 1: True}, dict(out)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def _graph_worker(rank, world, port, out, cfg=None):
    """bench.py's N-rank graph path: forward + backward captured into a HIP graph on the prefetched metadata,
    gradients as views of one flat buffer (dp.GradSync), one all-reduce + Adam eagerly after the replay.
    cfg: m, reps, scale, scenes (per rank) and oracle (rank 0 also checks the per-point features of one of
    its scenes against the fp64 oracle under shared ReLU decisions, at the 1e-4 bar)."""
    cfg = dict(dict(m=16, reps=2, scale=20, scenes=2, oracle=False), **(cfg or {}))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "3d-weakly-supervised-semantic-segmentation_amd"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import torch.nn.functional as F
    import sparseconvnet as scn
    from sparseconvnet import metadata as scn_meta
    from wsss3d import EasyDict, MODEL_REGISTRY, dp
    from wsss3d.synthetic import make_batch

    try:
        r, w, _, dev = dp.init_from_env("cuda", backend="gloo", device_index=0)
        pc = EasyDict(name="SparseConvUNet", m=cfg["m"], dimension=3, full_scale=4096, block_reps=cfg["reps"],
                      residual_blocks=True)
        cls, _ = MODEL_REGISTRY.get("MultiLabel")
        torch.manual_seed(0)
        local = cls(pc).to(dev)
        torch.manual_seed(0 if r == 0 else 7)  # rank 1 differs: GradSync must broadcast rank 0's parameters
        model = cls(pc).to(dev)
        gsync = dp.GradSync(model, dev)
        ok = all(torch.equal(p, q) for p, q in zip(model.parameters(), local.parameters()))
        bs = [make_batch(cfg["scenes"], cfg["scale"], seed=10 * r + k) for k in range(2)]
        xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
                       batch_offsets=b["batch_offsets"]) for b in bs]
        ys = [torch.from_numpy(b["scene_labels"]).to(dev) for b in bs]

        def loss_of(net, k):
            logits, _ = net((xs[k], None), istrain=True)
            return F.multilabel_soft_margin_loss(logits, ys[k])

        model.zero_grad(set_to_none=False)
        loss_of(model, 0).backward()         # records the rulebook plan
        torch.cuda.synchronize()
        assert scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False) is not None
        ev = scn_meta.prefetch_event(dev)
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        with torch.cuda.stream(cap):
            g.capture_begin(capture_error_mode="relaxed")
            model.zero_grad(set_to_none=False)
            loss_of(model, 1).backward()
            g.capture_end()
        assert scn_meta.captured_metadata()
        gsync.check_views()
        cur = torch.cuda.current_stream(dev)
        cur.wait_event(ev)
        g.replay()
        gsync.average()
        loss_of(local, 1).backward()
        for (k, p), q in zip(model.named_parameters(), local.parameters()):
            gl = q.grad.clone()
            dist.all_reduce(gl)
            gl /= w
            if not torch.allclose(p.grad, gl, rtol=1e-6, atol=1e-9):
                ok = False
                print(f"rank {r}: grad {k} differs by {(p.grad - gl).abs().max().item():.3e}", flush=True)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
        opt.step()
        flat = torch.cat([p.detach().flatten() for p in model.parameters()])
        ref = flat.clone()
        dist.broadcast(ref, 0)
        ok &= torch.equal(flat, ref)
        torch.cuda.synchronize()
        del g
        if cfg["oracle"] and r == 0:  # one whole scene of this rank's batch against the fp64 oracle
            from oracle.encoders import OracleEncoder
            from oracle.parity import run_shared_masks
            b0 = bs[1]
            n0 = int(b0["batch_offsets"][1])
            c0 = torch.from_numpy(b0["coords"][:n0])
            f0 = torch.from_numpy(b0["feats"][:n0])
            enc = model.pc_encoder
            oref = OracleEncoder("SparseConvUNet", m=cfg["m"], block_reps=cfg["reps"], residual_blocks=True).double()
            oref.load_state_dict({k: v.double().cpu() for k, v in enc.state_dict().items()})
            with torch.no_grad():
                og, oo, st = run_shared_masks(enc, oref, EasyDict(coords=c0.to(dev), feature=f0.to(dev),
                                                                  batch_offsets=[0, n0]),
                                              dict(coords=c0, feature=f0.double(), batch_offsets=[0, n0]),
                                              istrain=False)
            err = (og.double().cpu() - oo).abs().max().item()
            lim = 1e-4 * max(1.0, oo.abs().max().item())
            print(f"rank 0: scene 0 ({n0} points) per-point features max err {err:.3e} (bar {lim:.3e}), "
                  f"flip margin {st['max_flip_margin']:.2e}", flush=True)
            ok &= err <= lim and st["max_flip_margin"] < 1e-4
        out[rank] = bool(ok)
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        out[rank] = f"{type(e).__name__}: {e}"
        raise


def _run_graph_world2(cfg=None, timeout=300):
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    out = manager.dict()
    port = _free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, out, cfg)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert dict(out) == {0: True, 1: True}, dict(out)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_graph_dp_world2_hip_model():
    _run_graph_world2()


@pytest.mark.timeout(900)
def test_c4_per_rank_workload_graph_dp():
    """BASELINE configs[3] per-rank workload (SparseConvUNet m=32, block_reps=2, residual, scale 50 = 2 cm,
    5 whole scenes per rank) through bench.py's N-rank graph path on two ranks sharing cuda:0 over gloo:
    averaged gradients = the mean of the ranks' local gradients, parameters equal after Adam, and rank 0's
    per-point features of one of its scenes within 1e-4 of the fp64 oracle."""
    _run_graph_world2(dict(m=32, reps=2, scale=50, scenes=5, oracle=True), timeout=600)


def _overlap_worker(port, out):
    """One-rank RCCL group: the bucket all-reduces of dp.GradSync(overlap=True) captured into the step's graph
    (issued from post-accumulate-grad hooks during the captured backward) must leave exactly the local
    gradients (a one-rank mean) after the replay, bit for bit."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "3d-weakly-supervised-semantic-segmentation_amd"), root):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import torch.nn.functional as F
    import sparseconvnet as scn
    from sparseconvnet import metadata as scn_meta
    from wsss3d import EasyDict, MODEL_REGISTRY, dp
    from wsss3d.synthetic import make_batch
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        pc = EasyDict(name="SparseConvUNet", m=16, dimension=3, full_scale=4096, block_reps=2, residual_blocks=True)
        cls, _ = MODEL_REGISTRY.get("MultiLabel")
        torch.manual_seed(0)
        local = cls(pc).to(dev)
        torch.manual_seed(0)
        model = cls(pc).to(dev)
        gs = dp.GradSync(model, dev, overlap=True, bucket_mb=0.25)
        assert gs.overlap and len(gs.buckets) >= 3
        bs = [make_batch(2, 20, seed=k) for k in range(2)]
        xs = [EasyDict(coords=torch.from_numpy(b["coords"]).to(dev), feature=torch.from_numpy(b["feats"]).to(dev),
                       batch_offsets=b["batch_offsets"]) for b in bs]
        ys = [torch.from_numpy(b["scene_labels"]).to(dev) for b in bs]

        def loss_of(net, k):
            logits, _ = net((xs[k], None), istrain=True)
            return F.multilabel_soft_margin_loss(logits, ys[k])

        model.zero_grad(set_to_none=False)
        loss_of(model, 0).backward()
        torch.cuda.synchronize()
        assert scn.prefetch_metadata(model, xs[1].coords, wait_for_producer=False) is not None
        ev = scn_meta.prefetch_event(dev)
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        with torch.cuda.stream(cap):
            g.capture_begin(capture_error_mode="relaxed")
            model.zero_grad(set_to_none=False)
            gs.begin()
            loss_of(model, 1).backward()
            gs.join()
            g.capture_end()
        assert scn_meta.captured_metadata()
        torch.cuda.current_stream(dev).wait_event(ev)
        g.replay()
        loss_of(local, 1).backward()
        torch.cuda.synchronize()
        ok = all(torch.equal(p.grad, q.grad) for p, q in zip(model.parameters(), local.parameters()))
        del g
        out[0] = bool(ok)
        dist.destroy_process_group()
    except Exception as e:
        out[0] = f"{type(e).__name__}: {e}"
        raise


def test_grad_overlap_captured_rccl():
    ctx = mp.get_context("spawn")
    manager = ctx.Manager()
    out = manager.dict()
    p = ctx.Process(target=_overlap_worker, args=(_free_port(), out))
    p.start()
    p.join(timeout=240)
    if p.is_alive():
        p.kill()
    assert dict(out) == {0: True}, dict(out)


def test_bench_graph_path_over_rccl():
    """The exact code path the driver's multi-GPU bench runs (HIP-graph steps, dp.GradSync's all-reduce over
    RCCL between replays, eager Adam), on a one-rank RCCL group (BENCH_DP_SELFTEST): a small workload must
    complete and report the RCCL exchange."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_DP_SELFTEST="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1", "--no-cpu",
                        "--batch", "2", "--scale", "20", "--family-steps", "1"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["config"]["comm_backend"] == "nccl"
    assert d["config"]["grad_exchange"] and "captured" in d["config"]["grad_exchange"]
    assert "HIP graph" in d["config"]["launch"]
    assert d["value"] > 0
