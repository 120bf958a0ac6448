"""Micro-benchmark: production msp_conv_tile against the dense row-group form
(msp_debug_conv_nbr: neighbour map, register accumulators) on the headline
batch's real submanifold rulebooks.  Prints time, TF/s (algorithmic) and the
max error of each against an fp64 evaluation on a row subset (relative to
the subset's max |out|).
Usage: python scripts/kbench_nbr.py  (env LEVELS, FIRST_LEVEL, NBR = "nt:g,...", FLIP)."""
import os, sys, ctypes
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, ops
from sparseconvnet._lib import ptr
from wsss3d.synthetic import make_batch
lib = _lib.load()
P, I, I64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
fn = lib.msp_debug_conv_nbr
fn.restype = I64
fn.argtypes = [I, I, P, I, P, I, I, I, P, P, I64, P, P, SZ, P]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "4"))
first = int(os.environ.get("FIRST_LEVEL", "0"))
flip = int(os.environ.get("FLIP", "0"))
sizes = [4096 >> i for i in range(n_lv)]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
s = _lib.stream()
# nt:g[:ordered]  (ordered 1 = rows in SubmRules.dense_order's mask-sorted order)
VAR = [tuple([int(v) for v in e.split(":")] + [0, 0, 1][len(e.split(":")):]) for e in
       os.environ.get("NBR", "0:0:1,0:0:0").split(",")]
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
    print(f"L{L} V={V} R={rules.n_rules}", flush=True)
    rows = torch.arange(min(NSUB, V), device="cuda")
    nb = rules.nbr[:, :len(rows)].long()
    for cin, cout in ((c, c), (2 * c, c), (c, 2 * c)):
        torch.manual_seed(L)
        x = torch.randn(V, cin, device="cuda")
        wt = torch.randn(27, cout, cin, device="cuda") * (1.0 / (27 * cin) ** 0.5)
        flops = 2.0 * rules.n_rules * cin * cout
        x64 = torch.cat([x.double(), torch.zeros(1, cin, device="cuda", dtype=torch.float64)])
        g64 = x64[torch.where(nb >= 0, nb, V)]
        w64 = wt.double().flip(0) if flip else wt.double()
        ref = torch.einsum("onc,odc->nd", g64, w64)
        scale = ref.abs().max().item()
        f = lambda: ops.conv_tile(x, wt, 27, flip, cout, rules, V)
        ms = timeit(f)
        out = f()
        err = (out[:len(rows)].double() - ref).abs().max().item() / scale
        print(f"   {cin:3d}->{cout:3d} tile (production) {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF  err {err:.2e}", flush=True)
        prod = out.clone()
        perm, nbr_p = rules.dense_order()
        for nt, gg, ordered in VAR:
            if nt and (cout // 16) % nt:
                continue
            o2 = torch.empty(V, cout, device="cuda")
            mp, pp = (nbr_p, ptr(perm)) if ordered else (rules.nbr, None)
            need = fn(nt, gg, ptr(x), cin, ptr(wt), 27, flip, cout, ptr(mp), pp, V, ptr(o2), None, 0, s)
            ws = torch.empty(need // 4 + 1, device="cuda")
            args = (nt, gg, ptr(x), cin, ptr(wt), 27, flip, cout, ptr(mp), pp, V, ptr(o2), ptr(ws), int(need), s)

            def fx(args=args):
                rc = fn(*args)
                assert rc == 0, lib.msp_last_error()
            ms = timeit(fx)
            err = (o2[:len(rows)].double() - ref).abs().max().item() / scale
            dprod = ((o2 - prod).abs().max() / prod.abs().max()).item()
            print(f"   {cin:3d}->{cout:3d} nbr nt{nt} g{gg} o{ordered}     {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF  err {err:.2e}"
                  f"  vs prod {dprod:.1e}", flush=True)
