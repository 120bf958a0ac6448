"""What the device does at each graph replay's start: from a rocprofv3 kernel trace (+ memory-copy / HIP API traces
when present), per step: the last optimizer kernel's end, the first kernel of the next step, the second kernel, and
every memory copy or HIP API call that falls inside those windows.
Usage: step_boundary.py <prof dir>"""
import csv
import glob
import os
import sys

d = sys.argv[1]


def load(pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60], r["Stream_Id"])
            for r in load("*kernel_trace.csv"))
cp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "?")),
             r.get("Bytes", r.get("Size", "?"))) for r in load("*memory_copy_trace.csv"))
api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function", r.get("Operation", "?")))
             for r in load("*hip_api_trace.csv"))
t0 = ks[0][0]
s0 = [k for k in ks if k[3] == ks[[i for i, k in enumerate(ks) if "split_images" in k[2]][0]][3]]
firsts = [i for i, k in enumerate(s0) if "split_images" in k[2]]


def inside(lst, a, b):
    return [x for x in lst if x[1] > a and x[0] < b]


for i in firsts[1:]:
    prev, first, second = s0[i - 1], s0[i], s0[i + 1]
    print(f"step at {(first[0] - t0) / 1e6:10.3f} ms: idle before {(first[0] - prev[1]) / 1e3:8.1f} us "
          f"(after {prev[2][:40]}), first kernel {(first[1] - first[0]) / 1e3:6.1f} us, "
          f"gap to second {(second[0] - first[1]) / 1e3:7.1f} us ({second[2][:30]})")
    for a, b, what in ((prev[1], first[0], "before"), (first[1], second[0], "after first")):
        for x in inside(cp, a, b):
            print(f"    copy {what}: {(x[0] - t0) / 1e6:.3f} +{(x[1] - x[0]) / 1e3:.1f} us {x[2]} {x[3]}")
        other = [k for k in inside(ks, a, b) if k[3] != first[3]]
        if other:
            print(f"    {len(other)} other-stream kernels {what}, e.g. {other[0][2][:40]}")
        for x in inside(api, a, b)[:6]:
            print(f"    api {what}: {(x[0] - t0) / 1e6:.3f} +{(x[1] - x[0]) / 1e3:.1f} us {x[2]}")
