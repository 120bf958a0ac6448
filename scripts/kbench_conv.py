"""Micro-benchmark of msp_conv_tile on the headline batch's real rulebooks
(levels 0-LEVELS) for tile heights 64 / 128 / 256 and the kernel forms
(msp_debug_conv_tile variants), each checked against the 64-row production
result.  Usage: python scripts/kbench_conv.py  (env LEVELS, VARIANTS)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, metadata
from sparseconvnet._lib import ptr
from wsss3d.synthetic import make_batch
lib = _lib.load()
P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
fn = lib.msp_debug_conv_tile
fn.restype = I
fn.argtypes = [I, I, P, I, P, I, I, I, I, P, P, P, P, I64, P, P, P]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "4"))
sizes = [4096 >> i for i in range(n_lv)]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
s = _lib.stream()
# (label, tile_rows, abl, nt); abl None = production msp_conv_tile
VARIANTS = [
    ("prod64", 64, None, 0), ("prod128", 128, None, 0),
    ("t7-128-nt4-abl1", 128, 68, 4), ("t7-128-nt4-abl2", 128, 69, 4), ("t7-128-nt4-abl7", 128, 74, 4),
] + [(f"t7-128-nt{n}-s{k}", 128, 80 + k, n) for n in (1, 2, 3, 4) for k in (1, 2, 4, 8)]
sel = os.environ.get("VARIANTS")
if sel:
    VARIANTS = [v for v in VARIANTS if v[0] in sel.split(",")]


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
    if L < int(os.environ.get("FIRST_LEVEL", "0")):
        continue
    lvl = meta.level(size)
    rules = lvl.subm_rules(3)
    V = lvl.n
    c = 32 * (L + 1)
    if os.environ.get("SQUARE_ONLY"):
        pass
    books = {}
    for tr in (64, 128, 256):
        books[tr] = metadata.tile_rulebook(rules.nbr, 27, V, "cuda", s, tile_rows=tr)
    effs = " ".join(f"T{tr}:{rules.n_rules / (bk['n_chunks'] * 16):.2f}" for tr, bk in books.items())
    print(f"L{L} V={V} R={rules.n_rules} chunk eff {effs}", flush=True)
    for cin, cout in (((c, c),) if os.environ.get("SQUARE_ONLY") else ((c, c), (2 * c, c))):
        x = torch.randn(V, cin, device="cuda")
        wt = torch.randn(27, cout, cin, device="cuda") * 0.05
        flops = 2.0 * rules.n_rules * cin * cout
        ref = None
        for label, tr, abl, nt in VARIANTS:
            tl = books[tr]
            out = torch.empty(V, cout, device="cuda")
            if abl is None:
                wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(V), 27, cin, cout, tr))
                ws = torch.empty(max(wsb // 4, 1), device="cuda")
                f = lambda: _lib.call("msp_conv_tile", ptr(x), cin, ptr(wt), 27, 0, cout, tr, ptr(tl["tile_start"]),
                                      ptr(tl["chunk_off"]), ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out),
                                      ptr(ws), wsb, s)
            else:
                if (cout // 16) % nt:
                    continue
                ws = torch.empty(8 * V * cout, device="cuda")
                args = (abl, nt, ptr(x), cin, ptr(wt), 27, 0, cout, tr, ptr(tl["tile_start"]), ptr(tl["chunk_off"]),
                        ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), ptr(ws), s)

                def f(args=args):
                    rc = fn(*args)
                    assert rc == 0, lib.msp_last_error()
            try:
                ms = timeit(f)
            except (AssertionError, RuntimeError) as e:
                print(f"   {cin}->{cout} {label}: skipped ({e})")
                continue
            if ref is None:
                ref = out.clone()
                err = 0.0
            else:
                err = ((out - ref).abs().max() / ref.abs().max()).item()
            print(f"   {cin}->{cout} {label:16s} {ms:7.3f} ms  {flops / ms / 1e9:6.1f} TF(alg)  rel diff {err:.1e}",
                  flush=True)
