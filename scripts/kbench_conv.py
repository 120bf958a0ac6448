"""Micro-benchmark of msp_conv_tile on the headline batch's real rulebooks
(levels 0-2) with ablation variants (msp_debug_conv_tile)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib
from sparseconvnet._lib import ptr
from wsss3d.synthetic import make_batch
lib = _lib.load()
P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
fn = lib.msp_debug_conv_tile
fn.restype = I
fn.argtypes = [I, I, P, I, P, I, I, I, P, P, P, P, I64, P, P]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
sizes = [4096, 2048, 1024]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
variants = [int(v) for v in os.environ.get("ABL", "0,1,2,4,3,7").split(",")]
for L, (size, c) in enumerate(zip(sizes, [32, 64, 96])):
    lvl = meta.level(size)
    rules = lvl.subm_rules(3)
    tl = rules.tiles
    V = lvl.n
    x = torch.randn(V, c, device="cuda")
    wt = torch.randn(27, c, c, device="cuda") * 0.05
    out = torch.empty(V, c, device="cuda")
    flops = 2.0 * rules.n_rules * c * c
    print(f"L{L} V={V} R={rules.n_rules} chunks={tl['n_chunks']} eff={rules.n_rules / (tl['n_chunks'] * 16):.2f}")
    for nt in [int(v) for v in os.environ.get("NTS", "1,2,4").split(",")]:
        if (c // 16) % nt:
            continue
        for abl in variants:
            if abl == 48 and c > 64:
                continue
            args = (abl, nt, ptr(x), c, ptr(wt), 27, 0, c, ptr(tl["tile_start"]), ptr(tl["chunk_off"]),
                    ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), _lib.stream())
            for _ in range(3):
                assert fn(*args) == 0, lib.msp_last_error()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn(*args)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            extra = ""
            if abl == variants[0]:
                ref_out = out.clone()
            else:
                extra = f"  max|diff vs abl0|={(out - ref_out).abs().max().item():.2e}"
            print(f"   nt={nt} abl={abl}: {ms:.3f} ms  {flops / ms / 1e9:.1f} TF(alg){extra}")
