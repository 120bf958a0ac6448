"""conv_x6s's 16-row groups on the headline batch: how full they are and what three ways of filling them would give.

Input: the dumps scripts/kbench.py writes with X6S_DUMP=<dir>/gs (per level L: gs_L<L>.npy = rows per (tile, group,
offset) [tiles][8][27] and gs_mask_L<L>.npy = each tile row's 27-bit offset mask in the kernel's row order).
Prints per level: (1) the fill (rules / 16 x the (group, offset) pairs that run an MFMA step); (2) MFMA rows if the
pairs with at most T rows went to compacted 16-rule chunks; (3) the fill after a pairwise row-swap local search
between a tile's groups (400 sampled tiles); (4) the group-steps left if one MFMA step served several groups of a
wave's half whose rows for the offset sit at disjoint positions, with rows ordered for it (rare rows first, rotated
by 4 positions per group of the half).

Usage: python scripts/x6s_group_stats.py <dump dir>"""
import itertools
import os
import sys

import numpy as np

POP16 = np.array([bin(i).count("1") for i in range(1 << 16)], np.int64)


def pop(x):
    x = np.asarray(x, np.int64)
    return POP16[x & 0xFFFF] + POP16[(x >> 16) & 0xFFFF]


def tile_cost(m):
    return int(pop(np.bitwise_or.reduce(m.reshape(8, 16), axis=1)).sum())


def swap_search(m, passes=200):
    m = m.copy()
    grp = np.repeat(np.arange(8), 16)
    for _ in range(passes):
        g = m.reshape(8, 16)
        orr = np.bitwise_or.reduce(g, axis=1)
        pre = np.zeros((8, 17), np.int64)
        suf = np.zeros((8, 17), np.int64)
        for i in range(16):
            pre[:, i + 1] = pre[:, i] | g[:, i]
            suf[:, 15 - i] = suf[:, 16 - i] | g[:, 15 - i]
        ex = (pre[:, :16] | suf[:, 1:17]).reshape(128)  # group's OR without the member
        delta = pop(ex[:, None] | m[None, :]) + pop(ex[None, :] | m[:, None]) - \
            pop(orr[grp])[:, None] - pop(orr[grp])[None, :]
        delta[grp[:, None] == grp[None, :]] = 0
        k = int(np.argmin(delta))
        if delta.flat[k] >= 0:
            break
        i, j = divmod(k, 128)
        m[i], m[j] = m[j], m[i]
    return m


def min_batches(ms, cache={}):
    ms = tuple(sorted(m for m in ms if m))
    if ms in cache:
        return cache[ms]
    n, best = len(ms), len(ms)
    for k in range(1, n):
        for asg in itertools.product(range(k), repeat=n):
            acc, ok = [0] * k, True
            for m, a in zip(ms, asg):
                if acc[a] & m:
                    ok = False
                    break
                acc[a] |= m
            if ok and len(set(asg)) == k:
                best = k
                break
        if best < n:
            break
    cache[ms] = best
    return best


def main():
    d = sys.argv[1]
    rng = np.random.default_rng(0)
    for L in range(8):
        f = os.path.join(d, f"gs_L{L}.npy")
        if not os.path.exists(f):
            continue
        g = np.load(f).astype(np.int64)
        act = g > 0
        rules, mf = g.sum(), act.sum() * 16
        line = [f"L{L}: fill {rules / mf:.3f}"]
        for T in (4, 6, 8):
            sp = act & (g <= T)
            spr = (g * sp).sum(axis=(1, 2))
            rows = (act & (g > T)).sum() * 16 + (np.ceil(spr / 16) * 16).sum()
            line.append(f"T={T}: rows x{rows / mf:.3f} (sparse rules {spr.sum() / rules:.3f})")
        masks = np.load(os.path.join(d, f"gs_mask_L{L}.npy")).astype(np.int64)
        nt = len(masks) // 128
        idx = rng.choice(nt, min(nt, 400), replace=False)
        r_ = sum(int(pop(masks[t * 128:(t + 1) * 128]).sum()) for t in idx)
        c0 = sum(tile_cost(masks[t * 128:(t + 1) * 128]) for t in idx)
        c1 = sum(tile_cost(swap_search(masks[t * 128:(t + 1) * 128])) for t in idx)
        line.append(f"swaps: fill {r_ / (16 * c0):.3f} -> {r_ / (16 * c1):.3f}")
        now = new = 0
        for t in idx:
            rows = masks[t * 128:(t + 1) * 128].reshape(8, 16).copy()
            for gi in range(8):
                r = rows[gi][np.argsort(pop(rows[gi]), kind="stable")]
                rows[gi] = np.roll(r, 4 * (gi // 2))
            for o in range(27):
                pm = (((rows >> o) & 1) << np.arange(16)).sum(1)
                for h in (0, 1):
                    ms = [int(pm[gi]) for gi in (h, h + 2, h + 4, h + 6)]
                    now += sum(1 for m in ms if m)
                    new += min_batches(ms)
        line.append(f"merged steps x{new / now:.3f}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
