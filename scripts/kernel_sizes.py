"""Per-launch-shape breakdown of a rocprofv3 kernel trace: for every kernel whose name contains one of the
given substrings, the dispatches grouped by (kernel, grid size) with count, mean and total duration, largest
total first.  Usage: kernel_sizes.py <kernel_trace.csv> <substr>[,<substr>...] [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
subs = sys.argv[2].split(",")
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    if any(s in name for s in subs):
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        agg[(name[:58], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
total = sum(sum(v) for v in agg.values())
print(f"{'kernel':58s} {'grid':>9s} {'calls':>6s} {'mean us':>9s} {'total ms':>9s}")
for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{name:58s} {grid:>9s} {len(v):6d} {sum(v) / len(v):9.1f} {sum(v) / 1e3:9.2f}")
print(f"total {total / 1e3:.2f} ms over {sum(len(v) for v in agg.values())} dispatches")
