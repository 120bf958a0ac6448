"""msp_conv_pairs micro-benchmark on the headline batch (8 synthetic scenes at scale 50, the m = 32 UNet's strided
relations): per level L -> L+1, the deconvolution forward (coarse 32(L+2) channels -> fine 32(L+1)) and the strided
convolution's backward-data (same shapes), which are the two users of the pair-list convolution.  Times the product
library and, through each lib/libmi3dsparse_exp*.so (scripts/build_exp.sh, e.g. EXP_FLAGS=-DMSP_PAIRS_RUN=0), the same
call through it, and checks the two outputs are bit-identical.  HIP events, median of N.

Usage: python scripts/kbench_pairs.py   env: N=20  SCENES=8  M=32"""
import ctypes
import glob
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
    libs = {"prod": _lib.load()}
    for exp in sorted(glob.glob(os.path.join(_lib.PKG_ROOT, "lib", "libmi3dsparse_exp*.so"))):
        e = ctypes.CDLL(exp)
        res, args = _lib.PROTOTYPES["msp_conv_pairs"]
        e.msp_conv_pairs.restype, e.msp_conv_pairs.argtypes = res, args
        libs[os.path.basename(exp)[len("libmi3dsparse_"):-3]] = e
    b = make_batch(int(os.environ.get("SCENES", "8")), 50, seed=1)
    t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).to(DEV), torch.from_numpy(b["feats"]).to(DEV)])
    meta = t.metadata
    s = _lib.stream()
    g = torch.Generator(device=DEV).manual_seed(0)
    tot = {k: 0.0 for k in libs}
    for L in range(6):
        size = 4096 >> L
        coarse, rules = meta.downsample(size, 2)
        p = rules.pairs
        fine_n = meta.level(size).n
        cin, cout = M * (L + 2), M * (L + 1)
        xc = torch.randn(coarse.n, cin, device=DEV, generator=g)
        wt = torch.randn(8, cout, cin, device=DEV, generator=g)  # [K][c_out][c_in]
        outs, row = {}, [f"L{L} fine {fine_n:8d} coarse {coarse.n:8d} {cin:3d}->{cout:3d} pairs {p.total:8d}"]
        for name, lib in libs.items():
            out = torch.empty(fine_n, cout, device=DEV)

            def f():
                rc = lib.msp_conv_pairs(ptr(xc), cin, ptr(wt), 8, cout, ptr(p.pair_out), ptr(p.pair_in),
                                        ptr(p.off_start), ptr(p.chunk_start), p.n_chunks, ptr(out), s)
                assert rc == 0, rc
            ms = timeit(f)
            tot[name] += ms
            outs[name] = out.clone()
            nbytes = 4 * (coarse.n * cin + fine_n * cout + 8 * cin * cout) + 8 * p.total
            row.append(f"{name} {1e3 * ms:7.1f}us {nbytes / ms / 1e6:6.0f} GB/s")
        if len(outs) > 1:
            row.append(f"bit-identical {all(torch.equal(outs['prod'], v) for v in outs.values())}")
        print("  ".join(row), flush=True)
    print("sum over levels (one call each):", "  ".join(f"{k} {1e3 * v:7.1f}us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
