#!/bin/bash
# Round-4: where the 1 ms before each replay goes.  Host timing with the build-event timestamps: default loop,
# worker-thread prefetch, high-priority prefetch stream.  Then the prefetch/graph tests (incl. the worker-thread one).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B C; do
  extra=""; [ $v = B ] && extra="--prefetch-thread 1"; [ $v = C ] && extra="--prefetch-priority 1"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu $extra > gpurun_out/bench_r04o_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04o_host_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04o_host_$v.log)"; grep "graph loop host\|device idle\|build done" gpurun_out/bench_r04o_host_$v.log | cut -c1-300
done
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_encoders.py -k "prefetch or graph or metadata" > gpurun_out/pytest_r04o.log 2>&1 || { tail -30 gpurun_out/pytest_r04o.log; exit 1; }
tail -2 gpurun_out/pytest_r04o.log
