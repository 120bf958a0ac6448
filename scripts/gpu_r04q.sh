#!/bin/bash
# Round-4: PairLists chunk starts computed on the device (no host-to-device copy in the prefetch) and the count
# reads' host wait measured (metadata.READ_STATS): host timing of the graph loop, default (A) and with the
# worker-thread prefetch (B); then the prefetch / graph tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B; do
  extra=""; [ $v = B ] && extra="--prefetch-thread 1"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu $extra > gpurun_out/bench_r04q_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04q_host_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04q_host_$v.log)"; grep "graph loop host\|device idle\|build done\|count reads" gpurun_out/bench_r04q_host_$v.log | cut -c1-200
done
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_encoders.py -k "prefetch or graph or metadata" > gpurun_out/pytest_r04q.log 2>&1 || { tail -30 gpurun_out/pytest_r04q.log; exit 1; }
tail -2 gpurun_out/pytest_r04q.log
