"""One line per run of an A/B (scripts/gpu_ab.sh / gpu_args_ab.sh logs): ms/step, device median, family ms/step.
Usage: ab_summary.py <log> [<log> ...]"""
import json
import sys

for p in sys.argv[1:]:
    lines = [l for l in open(p) if l.startswith('{"metric"')]
    if not lines:
        print(p, "no result")
        continue
    d = json.loads(lines[-1])
    fams = {k: round(v["ms"] / 5, 2) for k, v in d.get("roofline_families", {}).items() if isinstance(v, dict)}
    print(p.split("/")[-1], round(d["ms_per_step"], 2), round(d["ms_per_step_median"], 2), fams)
