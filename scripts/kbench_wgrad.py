"""Micro-benchmark of msp_conv_wgrad on the headline batch's real submanifold
pair lists (levels 0-3, c -> c and 2c -> c), x6 (bf16 split) form against the
f32-MFMA form (msp_debug_wgrad_f32), each checked against torch fp64."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g; g.add_path()
import torch
import sparseconvnet as scn
from sparseconvnet import ops, _lib
from wsss3d.synthetic import make_batch
b = make_batch(8, 50, seed=1)
t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).cuda(), torch.from_numpy(b["feats"]).cuda()])
meta = t.metadata
sizes = [4096, 2048, 1024, 512]
for s_ in sizes[:-1]:
    meta.downsample(s_, 2)
lib = _lib.load()
cases = [(L, size, ci, c) for L, (size, c) in enumerate(zip(sizes, [32, 64, 96, 128])) for ci in (c, 2 * c)]
lib.msp_debug_wgrad_blocks.argtypes = [_lib.I64]
BLOCKS = [int(v) for v in os.environ.get("BLOCKS", "0").split(",")]
MODES = [int(v) for v in os.environ.get("MODES", "0,1").split(",")]
lib.msp_debug_wgrad_abl(int(os.environ.get("ABL", "0")))
lib.msp_debug_wgrad_tile(int(os.environ.get("WA", "0")), int(os.environ.get("WB", "0")))  # forced dW tile
for (L, size, ci, c), mode, nb in [(cs, m, nb) for cs in cases for m in MODES for nb in BLOCKS]:
    lib.msp_debug_wgrad_f32(1 if mode == 1 else 0)
    lib.msp_debug_wgrad_blocks(nb)
    rules = meta.level(size).subm_rules(3)
    p = rules.pairs
    V = meta.level(size).n
    torch.manual_seed(L)
    x = torch.randn(V, ci, device="cuda")
    dy = torch.randn(V, c, device="cuda")
    # mode 2: banded form (msp_conv_wgrad_band), else the pair-list form (mode 1: f32 MFMA)
    fw = (lambda: ops.conv_wgrad_band(x, dy, p, 27, V)) if mode == 2 else \
        (lambda: ops.conv_wgrad(x, dy, p, p.pair_in, p.pair_out, 27))
    for _ in range(2):
        dw = fw()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fw()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    offs = p.off_start.cpu().tolist()
    pin, pout = p.pair_in.long(), p.pair_out.long()
    err = 0.0
    for o in range(27):
        s0, s1 = offs[o], offs[o + 1]
        ref = x[pin[s0:s1]].double().T @ dy[pout[s0:s1]].double()
        err = max(err, ((dw[o].double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item())
    flops = 2.0 * rules.n_rules * ci * c
    print(f"L{L} {ci:3d}->{c:3d} {['x6 ', 'f32', 'band'][mode]} blocks~{nb or 4096} V={V} R={rules.n_rules} "
          f"pieces={_lib.query('msp_wgrad_pieces', _lib.I64(p.total), 27, ci, c)}: {ms:.3f} ms "
          f"{flops / ms / 1e9:.1f} TF  max rel err {err:.2e}", flush=True)
