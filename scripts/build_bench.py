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

        def hash_and_map():
            lvl._hash = None
            table, cap = lvl.hash()
            nbr = torch.empty((27, max(n, 1)), dtype=torch.int32, device=DEV)
            _lib.call("msp_subm_map", _lib.ptr(lvl.keys), n, lvl.log2, lvl.size, 3, _lib.ptr(table), cap,
                      _lib.ptr(nbr), s)
            return nbr
        ms = timeit(hash_and_map)
        tot["hash+map"] = tot.get("hash+map", 0.0) + ms
        nbr = hash_and_map()
        w = torch.arange(nbr.numel(), device=DEV, dtype=torch.int64) % 1000003 + 1
        row.append(f"hash+map {1e3 * ms:7.1f}us (map checksum {int((nbr.reshape(-1).long() * w).sum())}, "
                   f"same as the level's rules: {bool(torch.equal(nbr, rules.nbr))})")
        for name, lists_only in (("local", False), ("lists", True)):
            ms = timeit(lambda: metadata.local_rulebook(rules.nbr, 27, n, rules.nbr.device, s, 128,
                                                        lists_only=lists_only))
            tot[name] = tot.get(name, 0.0) + ms
            row.append(f"{name} {1e3 * ms:7.1f}us")
        print("  ".join(row), flush=True)
    print("sum over levels:", "  ".join(f"{k} {1e3 * v:8.1f}us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
