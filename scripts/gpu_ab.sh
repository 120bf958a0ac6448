#!/bin/bash
# Interleaved end-to-end A/B on one box: bench.py on the product library (A) and on lib/libmi3dsparse_exp.so
# (B, scripts/build_exp.sh with EXP_FLAGS), ROUNDS times each, alternating; one JSON line per run in
# gpurun_out/ab_$TAG.log (prefixed A / B).  B_ENV="VAR=value ..." sets environment variables for the B runs
# only; B_LIB=0 keeps B on the product library (an environment-only A/B); B_ARGS: extra bench.py arguments
# for the B runs; B_ROOT: run B from another tree (e.g. a previous commit's build staged under ab_prev/, when
# the change spans the library and its Python side).
set -o pipefail
TAG=${TAG:-ab}
ROUNDS=${ROUNDS:-2}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
EXP=${EXP_LIB:-$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib/libmi3dsparse_exp.so}
: > gpurun_out/ab_$TAG.log
for i in $(seq 1 $ROUNDS); do
  for v in A B; do
    unset MI3DSPARSE_LIB
    [ $v = B ] && [ "${B_LIB:-1}" = 1 ] && export MI3DSPARSE_LIB=$EXP
    envs=""
    extra=""
    [ $v = B ] && envs="${B_ENV:-}" && extra="${B_ARGS:-}"
    root=.
    [ $v = B ] && [ -n "${B_ROOT:-}" ] && root=$B_ROOT && unset MI3DSPARSE_LIB
    (cd $root && env $envs timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 15 --warmup 5} $extra) \
      > gpurun_out/ab_${TAG}_$v$i.log 2>&1 || exit $?
    echo "$v $(grep '^{"metric"' gpurun_out/ab_${TAG}_$v$i.log)" >> gpurun_out/ab_$TAG.log
    python - "$v" gpurun_out/ab_${TAG}_$v$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1])
fams = {k: round(v["ms"] / 5, 2) for k, v in d.get("roofline_families", {}).items() if isinstance(v, dict)}
print(sys.argv[1], round(d["ms_per_step"], 2), round(d["ms_per_step_median"], 2), fams, flush=True)
PY
  done
done
