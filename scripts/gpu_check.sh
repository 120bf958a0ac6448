#!/bin/bash
# One GPU session: smoke, GPU parity tests, short bench.  Every GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
  && echo "gpu tests ok" \
  && timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 \
  && echo "bench ok"
rc=$?
tail -5 gpurun_out/smoke.log; tail -30 gpurun_out/pytest_gpu.log 2>/dev/null; tail -3 gpurun_out/bench.log 2>/dev/null
exit $rc
