"""Choose wgrad_x6c's offset deal table (csrc/msp_local.hip kX6cDeal, template DL 1) offline.

Input: the per-tile k-step counts per offset that scripts/kbench.py dumps with X6C_STATS=1 X6C_DUMP=<dir>/ks
(one ks_n<tiles>.npy per level, [tiles][32] int16).  A tile takes its slowest wave's k-steps (every tile ends at a
block barrier); the cost of a deal is, per level, the sum over tiles of that maximum over the mean, weighted by the
level's share of the step's wgrad_x6c time.  Local search (moves and swaps, at most 4 offsets per wave) from the
round-robin deal, with random restarts; prints the ratios per level and the packed table.

Usage: python scripts/x6c_deal_search.py <dump dir> [restarts]"""
import glob
import os
import sys

import numpy as np

# each level's share of wgrad_x6c time in the headline step (kernel_by_grid, round 6): levels 0..4
LEVEL_WEIGHT = [2.0, 4.0, 2.9, 1.6, 0.5]


def load(d):
    ks = sorted((np.load(f).astype(np.int64)[:, :27] for f in glob.glob(os.path.join(d, "ks_n*.npy"))),
                key=lambda a: -len(a))
    return ks[:len(LEVEL_WEIGHT)]  # levels by tile count, largest first


def ratios(ks, asg):
    m = np.zeros((27, 8))
    m[np.arange(27), asg] = 1
    return [float((k @ m).max(1).sum() / (k.sum() / 8)) for k in ks]


def cost(ks, asg):
    return sum(w * r for w, r in zip(LEVEL_WEIGHT, ratios(ks, asg)))


def search(ks, b):
    c0, better = cost(ks, b), True
    while better:
        better = False
        for o in range(27):
            for w in range(8):
                if w == b[o]:
                    continue
                if (b == w).sum() < 4:
                    cand = b.copy()
                    cand[o] = w
                    c = cost(ks, cand)
                    if c < c0 - 1e-9:
                        b, c0, better = cand, c, True
                        continue
                for o2 in np.where(b == w)[0]:
                    cand = b.copy()
                    cand[o], cand[o2] = b[o2], b[o]
                    c = cost(ks, cand)
                    if c < c0 - 1e-9:
                        b, c0, better = cand, c, True
                        break
    return b, c0


def main():
    ks = load(sys.argv[1])
    restarts = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rng = np.random.default_rng(1)
    rr = np.array([o % 8 for o in range(27)])
    best, bc = search(ks, rr)
    for _ in range(restarts):
        st = best.copy()
        for _ in range(5):
            i, j = rng.choice(27, 2, replace=False)
            st[i], st[j] = st[j], st[i]
        b, c = search(ks, st)
        if c < bc:
            best, bc = b, c
    print("round-robin", [round(r, 3) for r in ratios(ks, rr)])
    print("best       ", [round(r, 3) for r in ratios(ks, best)])
    packed = []
    for w in range(8):
        offs = [int(o) for o in np.where(best == w)[0]] + [0xFF] * 4
        packed.append(sum(o << (8 * i) for i, o in enumerate(offs[:4])))
    print("kX6cDeal = {" + ", ".join(f"0x{v:08x}u" for v in packed) + "}")


if __name__ == "__main__":
    main()
