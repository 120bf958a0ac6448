#!/bin/bash
# One GPU session: smoke, GPU parity tests, short bench.  Every GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
{ echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo;
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } \
  > gpurun_out/host.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
       > gpurun_out/pytest_gpu.log 2>&1 \
  && echo "gpu tests ok" \
  && timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 \
  && echo "bench ok"
rc=$?
cat gpurun_out/host.txt; tail -5 gpurun_out/smoke.log; tail -30 gpurun_out/pytest_gpu.log 2>/dev/null; tail -3 gpurun_out/bench.log 2>/dev/null
exit $rc
