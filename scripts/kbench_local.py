"""Micro-benchmark: the tile-local submanifold convolution (msp_conv_local) against the production gather
forms (msp_conv_tile / msp_conv_nbr) on the headline batch's real rulebooks.  Prints time, TF/s (algorithmic)
and the max error of each against an fp64 evaluation on a row subset (relative to the subset's max |out|),
plus the tile-local rulebook build time and its distinct-row statistics.
Usage: python scripts/kbench_local.py  (env LEVELS, M, FLIP = 0 (fwd layout [K][cin][cout]) / 1 (bwd-data))."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_; g_.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import _lib, ops
from wsss3d.synthetic import make_batch
lib = _lib.load()
import ctypes
lib.msp_debug_conv_local.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
lib.msp_debug_conv_local_abl.argtypes = [ctypes.c_int]
lib.msp_debug_conv_local_wp.argtypes = [ctypes.c_int]
lib.msp_debug_conv_local_ri.argtypes = [ctypes.c_int]
ABLS = [int(a) for a in os.environ.get("ABL", "").split(",") if a]  # ablation variants of local 2:1:0
# local variants "wr:order:nt[:persistent[:wp[:ri]]]" (env VARIANTS; wp = weight image, 3 pieces / 2 fp32; ri = 1:
# conv_x6s keeps the staged rows' indices in registers across input-channel slices)
VARS = [tuple(int(v) for v in e.split(":")) for e in os.environ.get("VARIANTS", "1:1:0,2:1:0,2:1:1,2:0:0").split(",")]
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
n_lv = int(os.environ.get("LEVELS", "4"))
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
    ms_meta = timeit(lambda: scn.metadata.local_rulebook(rules.nbr, 27, V, rules.nbr.device, _lib.stream(), 128), 3)
    lib.msp_debug_conv_local(-1, 1, -1)
    loc_sorted = scn.metadata.local_rulebook(rules.nbr, 27, V, rules.nbr.device, _lib.stream(), 128)
    lib.msp_debug_conv_local(-1, 0, -1)
    loc_key = scn.metadata.local_rulebook(rules.nbr, 27, V, rules.nbr.device, _lib.stream(), 128)
    lib.msp_debug_conv_local(-1, 1, -1)
    rules._locals[128] = loc = loc_sorted
    us = loc["u_start"][:loc["n_tiles"] + 1]
    cnt = (us[1:] - us[:-1]).float()
    print(f"L{L} V={V} R={rules.n_rules} tiles={loc['n_tiles']} U/T mean {cnt.mean().item() / 128:.2f} "
          f"max {loc['max_u']} over-cap tiles {(cnt > 383).float().mean().item() * 100:.2f}%  "
          f"local rulebook build {ms_meta:.3f} ms", flush=True)
    c = int(os.environ.get("M", "32")) * (L + 1)
    rows = torch.arange(min(NSUB, V), device="cuda")
    nb = rules.nbr[:, :len(rows)].long()
    for cin, cout in ((c, c), (2 * c, c), (c, 2 * c)):
        torch.manual_seed(L)
        x = torch.randn(V, cin, device="cuda")
        w = torch.randn(27, cin, cout, device="cuda") * (1.0 / (27 * cin) ** 0.5)  # module layout [K][cin][cout]
        flops = 2.0 * rules.n_rules * cin * cout
        x64 = torch.cat([x.double(), torch.zeros(1, cin, device="cuda", dtype=torch.float64)])
        g64 = x64[torch.where(nb >= 0, nb, V)]
        if flip_bwd:   # bwd-data form: weights given [K][cout][cin] with the offset flipped
            wt = w.transpose(1, 2).contiguous()
            ref = torch.einsum("onc,odc->nd", g64, wt.double().flip(0))
            flip = 1
        else:
            wt = w
            ref = torch.einsum("onc,ocd->nd", g64, w.double())
            flip = 2
        scale = ref.abs().max().item()
        res = []
        for name, var in [("gather", None)] + [("local" + ":".join(map(str, v)), v) for v in VARS]:
            ops.CONV_LOCAL = var is not None
            if var is not None:
                lib.msp_debug_conv_local(var[0], -1, var[2])
                lib.msp_debug_conv_local_abl(-2 if len(var) > 3 and var[3] else -1)
                lib.msp_debug_conv_local_wp(var[4] if len(var) > 4 else 3)
                lib.msp_debug_conv_local_ri(var[5] if len(var) > 5 else 3)
                rules._locals[128] = loc_sorted if var[1] else loc_key
            f = lambda: ops.conv_tile(x, wt, 27, flip, cout, rules, V)
            ms = timeit(f)
            out = f()
            err = (out[:len(rows)].double() - ref).abs().max().item() / scale
            res.append(f"{name} {ms:6.3f} {flops / ms / 1e9:5.1f}TF {err:.0e}")
        for abl in ABLS:
            lib.msp_debug_conv_local(2, -1, 0)
            rules._locals[128] = loc_sorted
            lib.msp_debug_conv_local_abl(-1)
            lib.msp_debug_conv_local_abl(abl)
            ops.CONV_LOCAL = True
            ms = timeit(lambda: ops.conv_tile(x, wt, 27, flip, cout, rules, V))
            res.append(f"abl{abl} {ms:6.3f}")
            lib.msp_debug_conv_local_abl(0)
        print(f"   {cin:3d}->{cout:3d}  " + "  ".join(res), flush=True)
        lib.msp_debug_conv_local(2, 1, 0)
        lib.msp_debug_conv_local_abl(-3)
        lib.msp_debug_conv_local_wp(3)
        lib.msp_debug_conv_local_ri(3)
        rules._locals[128] = loc_sorted
ops.CONV_LOCAL = True
