"""Micro-benchmark: production msp_conv_tile (f32 MFMA) against the x6 form
(bf16 MFMA on exact three-piece splits, msp_debug_conv_x6) on the headline
batch's real submanifold rulebooks, levels 0..LEVELS-1.  Prints time, TF/s
(algorithmic) and the max error of each against an fp64 evaluation of the
same convolution on a row subset (relative to the subset's max |out|).
Usage: python scripts/kbench_x6.py  (env LEVELS, X6 = "nt:ks,..." variants)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, metadata
from sparseconvnet._lib import ptr
from wsss3d.synthetic import make_batch
lib = _lib.load()
P, I, I64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
fx6 = lib.msp_debug_conv_x6
fx6.restype = I64
fx6.argtypes = [I, I, I, I, I, P, I, P, I, I, I, P, P, P, P, I64, P, P, SZ, P]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "7"))
first = int(os.environ.get("FIRST_LEVEL", "0"))
sizes = [4096 >> i for i in range(n_lv)]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
s = _lib.stream()
# nt:ks:depth[:abl[:tile_rows]]  (abl: msp_conv_x6.hip ablation bits, timing only)
X6 = [tuple([int(v) for v in e.split(":")] + [0, 0, 0, 0, 128][len(e.split(":")):]) for e in
      os.environ.get("X6", "0:0:0,4:32:2,4:32:3,3:64:2,2:64:2").split(",")]
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
    if L < first:
        continue
    lvl = meta.level(size)
    rules = lvl.subm_rules(3)
    V = lvl.n
    c = int(os.environ.get("M", "32")) * (L + 1)
    tl = metadata.tile_rulebook(rules.nbr, 27, V, "cuda", s, tile_rows=128)
    print(f"L{L} V={V} R={rules.n_rules}", flush=True)
    rows = torch.arange(min(NSUB, V), device="cuda")
    nb = rules.nbr[:, :len(rows)].long()  # [27][n]
    for cin, cout in ((c, c), (2 * c, c)):
        if cout <= 32 and cin <= 64 and not os.environ.get("NARROW"):
            continue  # per-wave f32 form territory
        torch.manual_seed(L)
        x = torch.randn(V, cin, device="cuda")
        wt = torch.randn(27, cout, cin, device="cuda") * (1.0 / (27 * cin) ** 0.5)
        flops = 2.0 * rules.n_rules * cin * cout
        # fp64 reference on the first NSUB rows
        x64 = torch.cat([x.double(), torch.zeros(1, cin, device="cuda", dtype=torch.float64)])
        g64 = x64[torch.where(nb >= 0, nb, V)]  # [27][n][cin]
        ref = torch.einsum("onc,odc->nd", g64, wt.double())
        scale = ref.abs().max().item()
        wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(V), 27, cin, cout, 128))
        ws = torch.empty(max(wsb // 4, 1), device="cuda")
        out = torch.empty(V, cout, device="cuda")
        f = lambda: _lib.call("msp_conv_tile", ptr(x), cin, ptr(wt), 27, 0, cout, 128, ptr(tl["tile_start"]),
                              ptr(tl["chunk_off"]), ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out),
                              ptr(ws), wsb, s)
        ms = timeit(f)
        prod = out.clone()
        err = (out[:len(rows)].double() - ref).abs().max().item() / scale
        print(f"   {cin:3d}->{cout:3d} f32 tile7      {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF  err {err:.2e}", flush=True)
        for nt, ks, dp, abl, trx in X6:
            if nt and (cout // 16) % nt:
                continue
            tlx = tl if trx == 128 else metadata.tile_rulebook(rules.nbr, 27, V, "cuda", s, tile_rows=trx)
            args = [nt, ks, dp, abl, trx, ptr(x), cin, ptr(wt), 27, 0, cout, ptr(tlx["tile_start"]), ptr(tlx["chunk_off"]),
                    ptr(tlx["chunk_src"]), ptr(tlx["chunk_row"]), V, ptr(out), None, 0, s]
            need = fx6(*args)
            if need < 0:
                print(f"   {cin}->{cout} x6 nt{nt} ks{ks} d{dp}: {lib.msp_last_error()}")
                continue
            wsx = torch.empty(need // 4 + 1, device="cuda")
            args[17], args[18] = ptr(wsx), int(need)

            def fx(args=args):
                rc = fx6(*args)
                assert rc == 0, lib.msp_last_error()
            out.zero_()
            ms = timeit(fx)
            err = (out[:len(rows)].double() - ref).abs().max().item() / scale
            dprod = ((out - prod).abs().max() / prod.abs().max()).item()
            print(f"   {cin:3d}->{cout:3d} x6 nt{nt} ks{ks:2d} d{dp} a{abl:2d} t{trx} {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF  err {err:.2e}"
                  f"  vs f32 {dprod:.1e}", flush=True)
