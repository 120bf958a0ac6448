"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel and
counter, the mean value per dispatch.  Usage: pmc_summary.py DIR [FILTER]"""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: [0.0, set()])
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", r.get("Kernel-Name", "?")).split("(")[0]
        if filt and filt not in name:
            continue
        key = (name[:60], r["Counter_Name"])
        acc[key][0] += float(r["Counter_Value"])
        acc[key][1].add((f, r.get("Dispatch_Id", r.get("Correlation_Id"))))
for (name, ctr), (v, ds) in sorted(acc.items()):
    print(f"{name:60s} {ctr:28s} n={len(ds):5d} mean={v / max(len(ds), 1):.4g}")
