"""Per-step device occupancy from a rocprofv3 kernel trace of bench.py: steps are delimited by the fused tail
(msp::scene_final_kernel, once per forward); for each step the span, the merged busy time over all streams and
the idle time, plus the largest idle gaps.  Usage: step_gaps.py <kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]) for r in rows)
marks = [v[0] for v in iv if v[2].startswith("msp::scene_final_kernel")]
for k in range(1, len(marks)):
    s0, s1 = marks[k - 1], marks[k]
    sub = [v for v in iv if s0 <= v[0] < s1]
    busy, gaps, cs, ce, prev = 0, [], sub[0][0], sub[0][1], sub[0][2]
    for s, e, n in sub[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, prev, n))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        prev = n
    busy += ce - cs
    idle = sum(g[0] for g in gaps)
    big = sorted(gaps, reverse=True)[:3]
    print(f"step {k}: {(s1 - s0) / 1e6:6.2f} ms  busy {busy / 1e6:6.2f}  idle {idle / 1e6:5.2f} ms in {len(gaps)} gaps; "
          f"largest " + ", ".join(f"{g[0] / 1e3:.0f} us before {g[2][:30]}" for g in big))
