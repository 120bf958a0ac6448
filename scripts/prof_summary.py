"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"{'kernel':70s} {'calls':>6s} {'total ms':>9s} {'%':>5s} {'avg us':>8s}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r['Name'].split('(')[0][:70]
    print(f"{name:70s} {r['Calls']:>6s} {float(r['TotalDurationNs'])/1e6:9.2f} {100*float(r['TotalDurationNs'])/tot:5.1f} {float(r['AverageNs'])/1e3:8.1f}")
print(f"total kernel time {tot/1e6:.1f} ms")
