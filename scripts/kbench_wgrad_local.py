"""Micro-benchmark: the tile-local weight gradients (msp_conv_wgrad_local: dense 32-row steps;
msp_conv_wgrad_chunk: compacted chunks + transposing LDS reads) against the pair-list form (msp_conv_wgrad) on
the headline batch's real submanifold rulebooks, with the max error of each against an fp64 evaluation
(relative to max |dW|), and the chunk index build time.  Usage: python scripts/kbench_wgrad_local.py (env LEVELS,
M, FORMS = comma list of pairs,local,chunk)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, ops
from wsss3d.synthetic import make_batch
lib = _lib.load()
import ctypes
lib.msp_debug_wgrad_chunk.argtypes = [ctypes.c_int, ctypes.c_int]
ABLS = [int(a) for a in os.environ.get("ABL", "").split(",") if a]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "4"))
sizes = [4096 >> i for i in range(n_lv)]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)


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
    forms = os.environ.get("FORMS", "pairs,chunk").split(",")
    if "local" in forms:
        rules.local()
    tiles = rules.tiles_for(128)
    rules.local()

    def rebuild():
        rules._wchunk = None
        return rules.wgrad_index()
    ms_idx = timeit(rebuild, 3)
    idx = rules.wgrad_index()
    print(f"L{L} V={V} R={rules.n_rules} chunks(128)={tiles['n_chunks']} max distinct/tile "
          f"{rules.local()['max_u']}{' (over cap)' if idx is None else ''} index build {ms_idx:.3f} ms",
          flush=True)
    c = int(os.environ.get("M", "32")) * (L + 1)
    for cin, cout in ((c, c), (2 * c, c), (c, 2 * c)):
        torch.manual_seed(L)
        x = torch.randn(V, cin, device="cuda")
        dy = torch.randn(V, cout, device="cuda")
        flops = 2.0 * rules.n_rules * cin * cout
        p = rules.pairs
        nb = rules.nbr.long()
        ref = torch.empty(27, cin, cout, dtype=torch.float64, device="cuda")
        x64, dy64 = x.double(), dy.double()
        for o in range(27):
            m = nb[o] >= 0
            ref[o] = x64[nb[o][m]].t() @ dy64[m]
        scale = ref.abs().max().item()
        res = []
        fns = {"pairs": lambda: ops.conv_wgrad(x, dy, p, p.pair_in, p.pair_out, 27),
               "local": lambda: ops.conv_wgrad_local(x, dy, rules, 27),
               "chunk": lambda: ops.conv_wgrad_chunk(x, dy, rules, 27)}
        for nw in (8, 16):
            def fnw(nw=nw):
                lib.msp_debug_wgrad_chunk(nw, 0)
                return ops.conv_wgrad_chunk(x, dy, rules, 27)
            fns[f"chunk{nw}"] = fnw
        for abl in ABLS:
            def fab(abl=abl):
                lib.msp_debug_wgrad_chunk(8, abl)
                try:
                    return ops.conv_wgrad_chunk(x, dy, rules, 27)
                finally:
                    lib.msp_debug_wgrad_chunk(8, 0)
            fns[f"abl{abl}"] = fab
            forms = forms + [f"abl{abl}"] if f"abl{abl}" not in forms else forms
        for name, f in ((k, fns[k]) for k in forms):
            ms = timeit(f)
            err = (f().double() - ref).abs().max().item() / scale
            res.append(f"{name} {ms:6.3f} ms {flops / ms / 1e9:5.1f} TF err {err:.1e}")
        print(f"   {cin:3d}->{cout:3d}  " + "   ".join(res), flush=True)
