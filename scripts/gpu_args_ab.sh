#!/bin/bash
# Interleaved bench.py runs over argument sets on one box: ARGS_0, ARGS_1, ... (bench.py arguments, "-" for none),
# ROUNDS times each, alternating; one summary line per run in gpurun_out/args_$TAG.log.
set -o pipefail
TAG=${TAG:-args}
ROUNDS=${ROUNDS:-2}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/args_$TAG.log
for i in $(seq 1 $ROUNDS); do
  for k in 0 1 2 3; do
    var=ARGS_$k
    [ -n "${!var:-}" ] || continue
    a=${!var}; [ "$a" = "-" ] && a=""
    timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 15 --warmup 5} $a > gpurun_out/args_${TAG}_$k$i.log 2>&1 || exit $?
    python - "$k:$a" gpurun_out/args_${TAG}_$k$i.log <<'PY' | tee -a gpurun_out/args_$TAG.log
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1])
fams = {k: round(v["ms"] / 5, 2) for k, v in d.get("roofline_families", {}).items() if isinstance(v, dict)}
print(sys.argv[1], round(d["ms_per_step"], 2), round(d["ms_per_step_median"], 2), fams, flush=True)
PY
  done
done
