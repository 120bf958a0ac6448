"""Per-step kernel time from a rocprofv3 kernel trace of bench.py: steps are delimited by the fused tail
(msp::scene_final_kernel, once per forward); the kernels of steps [first, last) are summed by name and divided
by the step count (side-stream kernels overlap the main stream, so the sum exceeds the step's busy time).
Usage: step_kernels.py <kernel_trace.csv> [first last [top]]"""
import collections
import csv
import sys

def short(name):
    """Kernel name without its argument list; torch's elementwise kernels keep the functor they run."""
    base = name.split("(")[0]
    if base.startswith("void at::native::"):
        for key in ("FusedAdam", "CatArray", "direct_copy", "FillFunctor", "CUDAFunctor_add", "MulFunctor",
                    "BinaryFunctor", "reduce_kernel", "index", "sum", "neg"):
            if key in name:
                return "at::native::" + key
    return base[:90]


rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
marks = [v[0] for v in iv if v[2].startswith("msp::scene_final_kernel")]
first = int(sys.argv[2]) if len(sys.argv) > 2 else max(1, len(marks) // 4)
last = int(sys.argv[3]) if len(sys.argv) > 3 else len(marks) - 2
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
n = last - first
t_ms, calls = collections.Counter(), collections.Counter()
for s, e, name in iv:
    if marks[first] <= s < marks[last]:
        t_ms[name] += (e - s) / 1e6 / n
        calls[name] += 1 / n
print(f"steps {first}..{last} of {len(marks)}: kernel time {sum(t_ms.values()):.2f} ms/step, "
      f"span {(marks[last] - marks[first]) / 1e6 / n:.2f} ms/step")
print(f"{'ms/step':>8} {'calls':>6}  kernel")
for name, v in t_ms.most_common(top):
    print(f"{v:8.3f} {calls[name]:6.1f}  {name}")
