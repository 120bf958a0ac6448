#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no counters: those go
# in separate --pmc passes; ROCPROF_EXTRA adds trace domains, e.g. --memory-copy-trace).  Output under gpurun_out/prof_<tag>/.
set -o pipefail
TAG=${TAG:-r01}
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
# BENCH_ROOT: profile the bench of another tree (an A/B baseline staged under ab_prev/); outputs stay here
cd "${BENCH_ROOT:-$GRAFT_REPO_ROOT}"
timeout -k 10 600 rocprofv3 --kernel-trace ${ROCPROF_EXTRA:-} --stats --output-format csv -d $OUT/prof_${TAG} -o run -- \
  python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/prof_${TAG}.log 2>&1
cd "$GRAFT_REPO_ROOT"
rc=$?
find gpurun_out/prof_${TAG} -name "*stats*" | head; tail -2 gpurun_out/prof_${TAG}.log
exit $rc
