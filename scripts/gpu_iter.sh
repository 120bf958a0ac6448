# One iteration check on the GPU box: targeted GPU tests, the tile-local kbench (rulebook build times) and the
# default bench.  Usage: KEXPR="expr" bash scripts/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} \
  > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$KBENCH" ]; then
  LEVELS=5 VARIANTS=2:1:0 timeout -k 10 300 python scripts/kbench_local.py > gpurun_out/kb_$TAG.log 2>&1; rc=$?
  grep "^L" gpurun_out/kb_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1; rc=$?
tail -c 600 gpurun_out/bench_$TAG.log; exit $rc
