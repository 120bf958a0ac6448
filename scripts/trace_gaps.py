"""GPU occupancy of a rocprofv3 kernel trace: merges the kernel intervals of all streams and reports the busy
time, the idle gaps inside the traced span and the largest gaps (where the device waited on the host).
Usage: trace_gaps.py <kernel_trace.csv> [first_ns_fraction]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]) for r in rows)
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5  # skip the first part (warm-up, setup)
t0 = iv[0][0] + (iv[-1][1] - iv[0][0]) * frac
iv = [v for v in iv if v[0] >= t0]
busy, gaps, cur_s, cur_e, prev = 0, [], iv[0][0], iv[0][1], iv[0][2]
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = n
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
g = sum(x[0] for x in gaps)
print(f"span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {g / 1e6:.2f} ms ({100 * g / span:.1f} %), "
      f"{len(gaps)} gaps, {sum(1 for x in gaps if x[0] > 20000)} over 20 us")
for d, a, b in sorted(gaps, reverse=True)[:12]:
    print(f"  {d / 1e3:8.1f} us  after {a}  before {b}")
