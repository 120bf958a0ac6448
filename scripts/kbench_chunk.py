"""Micro-benchmark: the chunk-local submanifold convolution (msp_conv_chunk_local: 64-row tile rulebook, each
128-row unit's distinct input rows staged in LDS, LDS accumulators) against the forms the library takes without
it (per-wave gather tiles x6r, dense row groups x6g, tile-local x6s/x6l) on the headline batch's real rulebooks.
Prints time, TF/s (algorithmic) and the max error of each against fp64 on a row subset (relative to the subset's
max |out|), plus the chunk-local index build time.
Usage: python scripts/kbench_chunk.py  (env LEVELS, M, FLIP = 0 fwd layout / 1 bwd-data, DVS = value leads)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
import ctypes
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, ops
from wsss3d.synthetic import make_batch
lib = _lib.load()
lib.msp_debug_conv_chunk.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
ABLS = [int(a) for a in os.environ.get("ABL", "").split(",") if a]  # ablations of chunk4 (timing only)
DVS = [int(v) for v in os.environ.get("DVS", "2,3,4").split(",") if v]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "2"))
flip_bwd = int(os.environ.get("FLIP", "0"))
sizes = [4096 >> i for i in range(n_lv)]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
NSUB = 4096


def timeit(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for L, size in enumerate(sizes):
    lvl = meta.level(size)
    rules = lvl.subm_rules(3)
    V = lvl.n
    tiles = rules.tiles_for(64)
    ms_meta = timeit(lambda: scn.metadata.chunk_local_index(tiles, V, rules.nbr.device, _lib.stream()), 3)
    loc = rules.chunk_local()
    cnt = loc["u_cnt"][:loc["n_units"]].float()
    print(f"L{L} V={V} R={rules.n_rules} units={loc['n_units']} chunks={tiles['n_chunks']} "
          f"fill {rules.n_rules / (16 * tiles['n_chunks']):.3f} U/unit mean {cnt.mean().item():.1f} "
          f"max {int(cnt.max().item())} over-cap units {(cnt > loc['cap']).float().mean().item() * 100:.2f}%  "
          f"index build {ms_meta:.3f} ms", flush=True)
    c = int(os.environ.get("M", "32")) * (L + 1)
    rows = torch.arange(min(NSUB, V), device="cuda")
    nb = rules.nbr[:, :len(rows)].long()
    for cin, cout in ((c, c), (2 * c, c), (c, 2 * c)):
        torch.manual_seed(L)
        x = torch.randn(V, cin, device="cuda")
        w = torch.randn(27, cin, cout, device="cuda") * (1.0 / (27 * cin) ** 0.5)
        flops = 2.0 * rules.n_rules * cin * cout
        x64 = torch.cat([x.double(), torch.zeros(1, cin, device="cuda", dtype=torch.float64)])
        g64 = x64[torch.where(nb >= 0, nb, V)]
        if flip_bwd:
            wt = w.transpose(1, 2).contiguous()
            ref = torch.einsum("onc,odc->nd", g64, wt.double().flip(0))
            flip = 1
        else:
            wt = w
            ref = torch.einsum("onc,ocd->nd", g64, w.double())
            flip = 2
        scale = ref.abs().max().item()
        res = []
        for name, pref, dv in [("base", 0, 2)] + [(f"chunk{dv}", 1, dv) for dv in DVS]:
            lib.msp_debug_conv_chunk(dv, pref, 0)
            f = lambda: ops.conv_tile(x, wt, 27, flip, cout, rules, V)
            ms = timeit(f)
            out = f()
            err = (out[:len(rows)].double() - ref).abs().max().item() / scale
            res.append(f"{name} {ms:6.3f} {flops / ms / 1e9:5.1f}TF {err:.0e}")
        for abl in ABLS:
            lib.msp_debug_conv_chunk(4, 1, abl)
            ms = timeit(lambda: ops.conv_tile(x, wt, 27, flip, cout, rules, V))
            res.append(f"abl{abl} {ms:6.3f}")
        lib.msp_debug_conv_chunk(2, -1, 0)
        print(f"   {cin:3d}->{cout:3d}  " + "  ".join(res), flush=True)
