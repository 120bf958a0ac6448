"""Metadata-build micro-benchmark on the headline batch (8 synthetic scenes at scale 50, the m = 32 UNet's seven
levels): per level, the tile-local rulebook build (msp_tile_local: count + fill, with the row grouping and local
indices that conv_x6s reads, and lists only as the chunk-local weight gradient reads at level 0), HIP events,
median of N, the device otherwise idle.  The build runs on a side stream beside every training step, so its
kernel time is paid in the step.

Usage: python scripts/build_bench.py   env: N=7  SCENES=8"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import __graft_entry__ as g_  # noqa: E402
g_.add_path()
import torch  # noqa: E402
import sparseconvnet as scn  # noqa: E402
from sparseconvnet import _lib, metadata  # noqa: E402
from wsss3d.synthetic import make_batch  # noqa: E402

N = int(os.environ.get("N", "7"))
DEV = "cuda"


def timeit(f, n=N):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    b = make_batch(int(os.environ.get("SCENES", "8")), 50, seed=1)
    t = scn.InputLayer(3, 4096, mode=4)([torch.from_numpy(b["coords"]).to(DEV), torch.from_numpy(b["feats"]).to(DEV)])
    meta = t.metadata
    sizes = [4096 >> i for i in range(7)]
    for s_ in sizes[:-1]:
        meta.downsample(s_, 2)
    s = _lib.stream()
    tot = {}
    for L, size in enumerate(sizes):
        lvl = meta.level(size)
        rules = lvl.subm_rules(3)
        n = lvl.n
        row = [f"L{L} V={n:8d}"]
        for name, lists_only in (("local", False), ("lists", True)):
            ms = timeit(lambda: metadata.local_rulebook(rules.nbr, 27, n, rules.nbr.device, s, 128,
                                                        lists_only=lists_only))
            tot[name] = tot.get(name, 0.0) + ms
            row.append(f"{name} {1e3 * ms:7.1f}us")
        print("  ".join(row), flush=True)
    print("sum over levels:", "  ".join(f"{k} {1e3 * v:8.1f}us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
