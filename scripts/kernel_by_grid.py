"""Per-step time of the kernels whose name matches a pattern, split by grid size (a proxy for the level a call
serves), from a rocprofv3 kernel trace of bench.py.  Steps are delimited as in scripts/step_kernels.py.
Usage: kernel_by_grid.py <kernel_trace.csv> <substring> [<substring> ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
             int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), int(r.get("Workgroup_Size_X", 0) or 0))
            for r in rows)
marks = [v[0] for v in iv if v[2].startswith("msp::scene_final_kernel")]
first, last = max(1, len(marks) // 4), len(marks) - 2
n = last - first
agg = collections.defaultdict(lambda: [0.0, 0])
for s, e, name, grid, wg in iv:
    if marks[first] <= s < marks[last] and any(p in name for p in pats):
        k = (name[:60], grid // max(wg, 1))
        agg[k][0] += (e - s) / 1e6 / n
        agg[k][1] += 1
print(f"steps {first}..{last} of {len(marks)}")
print(f"{'ms/step':>8} {'calls':>6} {'us/call':>8} {'blocks':>8}  kernel")
tot = collections.Counter()
for (name, blocks), (ms, c) in sorted(agg.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    tot[name] += ms
    print(f"{ms:8.3f} {c / n:6.1f} {1e3 * ms / (c / n):8.1f} {blocks:8d}  {name}")
for name, ms in tot.most_common():
    print(f"{ms:8.3f}  total {name}")
