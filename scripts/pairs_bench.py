"""One-contribution-per-row kernels (deconvolution forward / strided backward-data, ``ops.conv_pairs``) on the
headline batch's real down rules (8 synthetic scenes at 2 cm, the m = 32 UNet's levels): the fp32 form
(``msp_conv_pairs``) against the split-bf16 form (``msp_conv_pairs_x6``), time (median of N launches, HIP events),
GB/s of the compulsory bytes (source rows, output rows, weights, pair lists) and the max error against fp64 on a
row subset.  Usage: python scripts/pairs_bench.py   env: LEVELS=0,1,2,3,4,5  N=20  M=32"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_  # noqa: E402
g_.add_path()
import torch  # noqa: E402
import sparseconvnet as scn  # noqa: E402
from sparseconvnet import _lib  # noqa: E402
from sparseconvnet._lib import ptr  # noqa: E402
from wsss3d.synthetic import make_batch  # noqa: E402

LEVELS = [int(v) for v in os.environ.get("LEVELS", "0,1,2,3,4,5").split(",")]
N = int(os.environ.get("N", "20"))
M = int(os.environ.get("M", "32"))
DEV = "cuda"


def timeit(f, n=N):
    for _ in range(3):
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


def main():
    b = make_batch(int(os.environ.get("SCENES", "8")), 50, seed=1)
    t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).to(DEV), torch.from_numpy(b["feats"]).to(DEV)])
    meta = t.metadata
    variants = [int(v) for v in os.environ.get("VARIANTS", "").split(",") if v]
    lib = _lib.load()
    exp = getattr(lib, "msp_exp_conv_pairs_x6", None)
    if exp is not None:
        import ctypes
        P, I, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        exp.restype = I
        exp.argtypes = [I, P, I, P, I, I, P, P, P, P, I64, P, P, ctypes.c_size_t, P]
    tot = {}
    for L in LEVELS:
        fine_size = 4096 >> L
        fine = meta.level(fine_size)
        coarse, rules = meta.downsample(fine_size, 2)
        p = rules.pairs
        cin, cout = M * (L + 2), M * (L + 1)
        K = 8
        torch.manual_seed(L)
        x = torch.randn(coarse.n, cin, device=DEV)
        wt = torch.randn(K, cout, cin, device=DEV)
        n_fine = fine.n
        nbytes = 4 * (coarse.n * cin + n_fine * cout + K * cin * cout) + 8 * p.total
        flops = 2.0 * p.total * cin * cout
        wsb = int(_lib.query("msp_conv_pairs_x6_workspace_size", K, cin, cout))
        ws = torch.empty(wsb // 4 + 4, device=DEV)

        def run(kind, variant=0):
            out = torch.empty(n_fine, cout, device=DEV)

            def f():
                if kind == "f32":
                    _lib.call("msp_conv_pairs", ptr(x), cin, ptr(wt), K, cout, ptr(p.pair_out), ptr(p.pair_in),
                              ptr(p.off_start), ptr(p.chunk_start), p.n_chunks, ptr(out), _lib.stream())
                elif kind == "x6":
                    _lib.call("msp_conv_pairs_x6", ptr(x), cin, ptr(wt), K, cout, ptr(p.pair_out), ptr(p.pair_in),
                              ptr(p.off_start), ptr(p.chunk_start), p.n_chunks, ptr(out), ptr(ws), wsb, _lib.stream())
                else:
                    rc = exp(variant, ptr(x), cin, ptr(wt), K, cout, ptr(p.pair_out), ptr(p.pair_in),
                             ptr(p.off_start), ptr(p.chunk_start), p.n_chunks, ptr(out), ptr(ws), wsb,
                             _lib.stream())
                    assert rc == 0, lib.msp_last_error()
            return f, out

        # fp64 on a subset of output rows
        pin, pout = p.pair_out.long(), p.pair_in.long()  # source (coarse) and output (fine) rows
        offs = torch.zeros(p.total, dtype=torch.long, device=DEV)
        os_ = p.off_start.long().tolist()
        for o in range(K):
            offs[os_[o]:os_[o + 1]] = o
        sel = torch.randperm(p.total, device=DEV)[:4096]
        ref = torch.einsum("nc,noc->no", x[pin[sel]].double(), wt[offs[sel]].double())
        forms = [("f32", 0), ("x6", 0)] + [("exp", v) for v in variants]
        line = []
        for kind, v in forms:
            f, out = run(kind, v)
            ms = timeit(f)
            err = (out[pout[sel]].double() - ref).abs().max().item() / ref.abs().max().item()
            name = kind if kind != "exp" else f"exp{v}"
            tot[name] = tot.get(name, 0.0) + ms
            line.append(f"{name} {ms * 1e3:7.1f} us {nbytes / ms / 1e6:6.0f} GB/s {flops / ms / 1e9:6.1f} TF/s "
                        f"err {err:.1e}")
        print(f"L{L} {cin}->{cout} pairs {p.total} src rows {coarse.n}: " + " | ".join(line), flush=True)
    print("total us: " + ", ".join(f"{k} {v * 1e3:.1f}" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
