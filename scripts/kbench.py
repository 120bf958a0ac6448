"""Kernel micro-benchmark on the headline batch's real rulebooks (BASELINE configs[2]: 8 synthetic scenes at
scale 50 = 2 cm, the m = 32 UNet's levels): every submanifold convolution form the library has, for the channel
pairs the network runs at each level (a -> a, 2a -> a forward; a -> 2a backward-data), and the weight-gradient
forms.  Prints time (median of N launches, HIP events), algorithmic TF/s (2 rules c_in c_out per rule) and the
max error of each against an fp64 evaluation on a row subset (relative to the subset's max |out|).

Usage: python scripts/kbench.py   env: LEVELS=0,1,2 (default 0-4)  PASSES=fwd,bwd,wgrad  FORMS=local,tile,nbr,...
       N=10 (timed launches)  SCENES=8"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_  # noqa: E402
g_.add_path()
import torch  # noqa: E402
import sparseconvnet as scn  # noqa: E402
from sparseconvnet import _lib, ops  # noqa: E402
from sparseconvnet._lib import ptr  # noqa: E402
from wsss3d.synthetic import make_batch  # noqa: E402

LEVELS = [int(v) for v in os.environ.get("LEVELS", "0,1,2,3,4").split(",")]
PASSES = os.environ.get("PASSES", "fwd,bwd,wgrad").split(",")
FORMS = os.environ.get("FORMS", "")
WFORMS = os.environ.get("WFORMS", "")
N = int(os.environ.get("N", "10"))
M = int(os.environ.get("M", "32"))
NSUB = 4096
DEV = "cuda"


def timeit(f, n=N):
    for _ in range(max(2, n // 2)):
        f()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        f()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def conv_forms(rules, V, cin, cout):
    """name -> f(x, wt, flip) for every form that applies (wt: [K][c_out][c_in], or [K][c_in][c_out] with flip 2)."""
    forms = {}

    def tile(x, wt, flip):
        tl = rules.tiles_for(128)
        out = torch.empty(V, cout, device=DEV)
        wsb = int(_lib.query("msp_conv_tile_workspace_size", _lib.I64(V), 27, cin, cout, 128))
        ws = torch.empty(max(wsb // 4, 1), device=DEV)
        _lib.call("msp_conv_tile", ptr(x), cin, ptr(wt), 27, flip, cout, 128, ptr(tl["tile_start"]),
                  ptr(tl["chunk_off"]), ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), ptr(ws), wsb,
                  _lib.stream())
        return out
    forms["tile"] = tile
    forms["local"] = lambda x, wt, flip: ops.conv_local(x, wt, 27, flip, cout, rules, V)

    def nbr(x, wt, flip):
        perm, nbr_p = rules.dense_order()
        return ops.conv_nbr(x, wt, 27, flip, cout, nbr_p, V, perm=perm)
    forms["nbr"] = nbr
    lib = _lib.load()
    if hasattr(lib, "msp_exp_conv_local") and cout % 32 == 0:  # the MSP_EXPERIMENTS build: conv_x6s variants
        import ctypes
        fn = lib.msp_exp_conv_local
        P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        fn.restype = I
        fn.argtypes = [I, P, I, P, I, I, I, I, P, P, P, P, P, I64, P, P, ctypes.c_size_t, P]

        def exp(variant):
            def f(x, wt, flip):
                loc = rules.local()
                out = torch.empty(V, cout, device=DEV)
                wsb = int(_lib.query("msp_conv_local_workspace_size", 27, cin, cout))
                ws = torch.empty(max(wsb // 4, 1), device=DEV)
                rc = fn(variant, ptr(x), cin, ptr(wt), 27, flip, cout, 128, ptr(loc["lidx"]), ptr(loc["u_start"]),
                        ptr(loc["u_rows"]), ptr(loc["perm"]), ptr(loc["wave_off"]), V, ptr(out), ptr(ws), wsb,
                        _lib.stream())
                if rc:
                    raise RuntimeError(lib.msp_last_error().decode())
                return out
            return f
        for v in [int(t) for t in os.environ.get("EXP_VARIANTS", "0,1").split(",") if t]:
            forms[f"x6s_v{v}"] = exp(v)
    if hasattr(lib, "msp_exp_conv_x6r") and cout <= 32 and cin <= 64:  # experiments build: per-wave tile variants
        import ctypes
        fx = lib.msp_exp_conv_x6r
        P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        fx.restype = I
        fx.argtypes = [I, P, I, P, I, I, I, I, P, P, P, P, I64, P, P, ctypes.c_size_t, P]

        def x6r(variant):
            tr = 64 if variant % 10 == 1 else 128

            def f(x, wt, flip):
                tl = rules.tiles_for(tr)
                out = torch.empty(V, cout, device=DEV)
                wsb = 27 * cout * ((cin + 31) // 32) * 32 * 6 + 1024 + (V * cin * 6 if variant >= 100 else 0)
                ws = torch.empty(max(wsb // 4, 1), device=DEV)
                rc = fx(variant, ptr(x), cin, ptr(wt), 27, flip, cout, tr, ptr(tl["tile_start"]), ptr(tl["chunk_off"]),
                        ptr(tl["chunk_src"]), ptr(tl["chunk_row"]), V, ptr(out), ptr(ws), wsb, _lib.stream())
                if rc:
                    raise RuntimeError(lib.msp_last_error().decode())
                return out
            return f
        for v in [int(t) for t in os.environ.get("X6R_VARIANTS", "30,31,20,21").split(",") if t]:
            forms[f"x6r_v{v}"] = x6r(v)
    if hasattr(ops, "conv_unit") and cout <= 64:
        forms["unit"] = lambda x, wt, flip: ops.conv_unit(x, wt, 27, flip, cout, rules, V)
    if FORMS:
        forms = {k: v for k, v in forms.items() if k in FORMS.split(",")}
    return forms


def x6c_balance(tiles):
    """wgrad_x6c's per-tile wave balance: k-steps (two chunks each) per (tile, offset), waves owning offsets
    w, w + 8, ...; a tile takes the slowest wave's k-steps.  Prints sum over tiles of (max wave) / (mean wave) and
    what a per-tile longest-first deal onto 8 waves (<= 4 offsets each) would give."""
    import numpy as np
    ts = tiles["tile_start"].cpu().numpy().astype(np.int64)
    co = tiles["chunk_off"].cpu().numpy().astype(np.int64)
    nt = len(ts) - 2  # tile_start carries the largest tile's chunk count after the total
    ts = ts[:nt + 1]
    tile_of = np.repeat(np.arange(nt), np.diff(ts))
    ch = np.zeros((nt, 32), np.int64)
    np.add.at(ch, (tile_of, co[:ts[-1]]), 1)
    ks = (ch + 1) // 2
    if os.environ.get("X6C_DUMP"):  # per-tile k-steps per offset, for choosing the offset deal offline
        np.save(os.environ["X6C_DUMP"] + f"_n{nt}.npy", ks.astype(np.int16))
    wave = ks.reshape(nt, 4, 8).sum(1)  # offset o = w + 8 a
    mx, mean = wave.max(1).sum(), ks.sum() / 8
    lpt = 0
    for t in range(nt):
        load = np.zeros(8, np.int64)
        cntw = np.zeros(8, np.int64)
        for o in np.argsort(-ks[t], kind="stable"):
            if ks[t, o] == 0:
                break
            cand = np.where(cntw < 4, load, 1 << 60)
            w = int(np.argmin(cand))
            load[w] += ks[t, o]
            cntw[w] += 1
        lpt += load.max()
    print(f"  x6c balance: k-steps {ks.sum()} mean/wave {mean:.0f}  fixed deal max {mx} ({mx / mean:.2f}x)  "
          f"per-tile LPT max {lpt} ({lpt / mean:.2f}x)  centre offset share {ks[:, 13].sum() / ks.sum():.3f}", flush=True)
    # per range (equal tile counts, R ranges): a range-wide deal (the rejected OB form) still waits per tile;
    # 'no barrier' = each wave's range total (the bound if waves never waited for each other inside a range)
    for R in sorted({max(1, 256 // s_) for s_ in (1, 4, 9, 16, 25)}):
        if R > nt:
            continue
        b_ = [t_ * nt // R for t_ in range(R + 1)]
        ob, nob, rng_mean = 0, 0, 0.0
        for r_ in range(R):
            blk = ks[b_[r_]:b_[r_ + 1]]
            tot = blk.sum(0)
            load = np.zeros(8, np.int64)
            cntw = np.zeros(8, np.int64)
            asg = {}
            for o in np.argsort(-tot, kind="stable"):
                if o >= 27:
                    continue
                w = int(np.argmin(np.where(cntw < 4, load, 1 << 60)))
                asg[o] = w
                load[w] += tot[o]
                cntw[w] += 1
            wv = np.zeros((len(blk), 8), np.int64)
            for o, w in asg.items():
                wv[:, w] += blk[:, o]
            ob = max(ob, wv.max(1).sum())
            nob = max(nob, blk.reshape(len(blk), 4, 8).sum(1).sum(0).max())
            rng_mean = max(rng_mean, blk.sum() / 8)
        print(f"    R={R}: slowest range: mean/wave {rng_mean:.0f}  range-LPT deal with per-tile waits {ob}  "
              f"fixed deal without waits {nob}", flush=True)


def main():
    b = make_batch(int(os.environ.get("SCENES", "8")), 50, seed=1)
    t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).to(DEV), torch.from_numpy(b["feats"]).to(DEV)])
    meta = t.metadata
    sizes = [4096 >> i for i in range(max(LEVELS) + 1)]
    for s_ in sizes[:-1]:
        meta.downsample(s_, 2)
    for L in LEVELS:
        lvl = meta.level(sizes[L])
        rules = lvl.subm_rules(3)
        V = lvl.n
        loc = rules.local()
        us = loc["u_start"][:loc["n_tiles"] + 1]
        cnt = (us[1:] - us[:-1]).float()
        tl = rules.tiles_for(128)
        fill = rules.n_rules / max(tl["n_chunks"] * 16, 1)
        print(f"L{L} V={V} R={rules.n_rules} ({rules.n_rules / V:.1f}/row) tiles={loc['n_tiles']} distinct rows "
              f"per tile {cnt.mean().item() / 128:.2f}x128 (max {loc['max_u']}) chunk fill {fill:.2f}", flush=True)
        if os.environ.get("X6C_STATS") == "1" and rules.wgrad_index() is not None:
            x6c_balance(rules.wgrad_index()["tiles"])
        if os.environ.get("X6S_DUMP") and "lidx" in loc:  # conv_x6s's rows per (tile, 16-row group, offset)
            import numpy as np
            nt_ = loc["n_tiles"]
            pres = (loc["lidx"][:, :nt_ * 128] != -1).view(27, nt_, 8, 16).sum(3)  # uint16 0xFFFF = absent
            np.save(os.environ["X6S_DUMP"] + f"_L{L}.npy", pres.permute(1, 2, 0).to(torch.uint8).cpu().numpy())
            bits = (loc["lidx"][:, :nt_ * 128] != -1).to(torch.int64)
            mask = (bits << torch.arange(27, device=DEV).view(27, 1)).sum(0)  # offset mask per tile row position
            np.save(os.environ["X6S_DUMP"] + f"_mask_L{L}.npy", mask.to(torch.int32).cpu().numpy())
        a = M * (L + 1)
        rows = torch.arange(min(NSUB, V), device=DEV)
        nb = rules.nbr[:, :len(rows)].long()
        shapes = []
        if "fwd" in PASSES:
            shapes += [("fwd", a, a), ("fwd", 2 * a, a)]
        if "bwd" in PASSES:
            shapes += [("bwd", a, a), ("bwd", a, 2 * a)]
        for pas, cin, cout in shapes:
            torch.manual_seed(L * 7 + cin + cout)
            x = torch.randn(V, cin, device=DEV)
            w = torch.randn(27, cin if pas == "fwd" else cout, cout if pas == "fwd" else cin, device=DEV)
            w *= 1.0 / (27 * cin) ** 0.5  # the module's layout [K][c_in][c_out] of the conv this pass belongs to
            flops = 2.0 * rules.n_rules * cin * cout
            x64 = torch.cat([x.double(), torch.zeros(1, cin, device=DEV, dtype=torch.float64)])
            g64 = x64[torch.where(nb >= 0, nb, V)]
            if pas == "fwd":  # forward: the module's weights as they are (flip bit 1)
                wt, flip = w, 2
                ref = torch.einsum("onc,ocd->nd", g64, w.double())
            else:  # backward-data: the same [K][c_out][c_in] tensor read as W^T with offsets mirrored (flip bit 0)
                wt, flip = w, 1
                ref = torch.einsum("onc,odc->nd", g64, w.double().flip(0))
            scale = ref.abs().max().item()
            res, best = [], {}
            forms = conv_forms(rules, V, cin, cout)
            for _ in range(2):  # two passes over the forms, the better of each form's medians (clock ramp)
                for name, f in forms.items():
                    try:
                        ms = timeit(lambda: f(x, wt, flip))
                        best[name] = min(best.get(name, ms), ms)
                    except Exception as e:  # a form that does not take this shape
                        best[name] = str(e)[:40]
            for name, f in forms.items():
                if isinstance(best[name], str):
                    res.append(f"{name} n/a ({best[name]})")
                    continue
                ms = best[name]
                out = f(x, wt, flip)
                err = (out[:len(rows)].double() - ref).abs().max().item() / scale
                res.append(f"{name} {ms:6.3f}ms {flops / ms / 1e9:6.1f}TF {err:.0e}")
            print(f"  {pas} {cin:3d}->{cout:3d}  " + "  ".join(res), flush=True)
        if "wgrad" in PASSES:
            for cin, cout in ((a, a), (2 * a, a), (a, 2 * a)):
                torch.manual_seed(L + cin * 3 + cout)
                x = torch.randn(V, cin, device=DEV)
                dy = torch.randn(V, cout, device=DEV)
                flops = 2.0 * rules.n_rules * cin * cout
                ref = torch.empty(27, cin, cout, dtype=torch.float64, device=DEV)
                nbl = rules.nbr.long()
                for o in range(27):
                    m = nbl[o] >= 0
                    ref[o] = x.double()[nbl[o][m]].t() @ dy.double()[m]
                scale = ref.abs().max().item()
                p = rules.pairs
                fs = {"pairs": lambda: ops.conv_wgrad(x, dy, p, p.pair_in, p.pair_out, 27)}
                if int(_lib.query("msp_wgrad_chunk_ok", _lib.I64(V), 27, cin, cout)) and rules.wgrad_index() is not None:
                    fs["chunk"] = lambda: ops.conv_wgrad_chunk(x, dy, rules, 27)
                lib = _lib.load()
                if "chunk" in fs and hasattr(lib, "msp_exp_wgrad_chunk"):  # MSP_EXPERIMENTS: wgrad_x6c variants
                    import ctypes
                    fn = lib.msp_exp_wgrad_chunk
                    P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
                    fn.restype = I
                    fn.argtypes = [I, P, I, P, I, I, I, P, P, P, P, P, I64, I64, P, P, P]

                    def wexp(variant, x=x, dy=dy, cin=cin, cout=cout):
                        def f():
                            idx = rules.wgrad_index()
                            tiles = idx["tiles"]
                            ranges = int(_lib.query("msp_wgrad_chunk_ranges", _lib.I64(V), cin, cout))
                            dw = torch.empty((27, cin, cout), device=DEV)
                            slab = torch.empty((ranges, 27, cin, cout), device=DEV)
                            rc = fn(variant, ptr(x), cin, ptr(dy), cout, 27, tiles["tile_rows"], ptr(tiles["tile_start"]),
                                    ptr(tiles["chunk_off"]), ptr(idx["chunk_lr"]), ptr(idx["u_start"]), ptr(idx["u_rows"]),
                                    V, ranges, ptr(slab), ptr(dw), _lib.stream())
                            if rc:
                                raise RuntimeError(lib.msp_last_error().decode())
                            return dw
                        return f
                    for v in [int(t) for t in os.environ.get("WEXP_VARIANTS", "0,1").split(",") if t]:
                        fs[f"x6c_v{v}"] = wexp(v)
                if WFORMS:
                    fs = {k: v for k, v in fs.items() if k in WFORMS.split(",")}
                if hasattr(ops, "conv_wgrad_unit"):
                    fs["unit"] = lambda: ops.conv_wgrad_unit(x, dy, rules, 27)
                res, first_x6c = [], None
                for name, f in fs.items():
                    try:
                        ms = timeit(f)
                        out = f()
                        err = (out.double() - ref).abs().max().item() / scale
                        same = ""
                        if name.startswith("x6c_v"):  # bit-identity against the first variant listed
                            if first_x6c is None:
                                first_x6c = out
                            else:
                                same = " =" if torch.equal(out, first_x6c) else " !="
                        res.append(f"{name} {ms:6.3f}ms {flops / ms / 1e9:6.1f}TF {err:.0e}{same}")
                    except Exception as e:
                        res.append(f"{name} n/a ({str(e)[:40]})")
                print(f"  wgrad {cin:3d}x{cout:3d}  " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
