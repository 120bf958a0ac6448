#!/bin/bash
# Round-4: is the 1 ms before each replay the compute stream's wait on the (long completed) build event?
# A = default, B = BENCH_SKIP_DONE_WAIT=1 (no wait issued when the event has completed).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B A2 B2; do
  envs="BENCH_HOST_TIMING=1"; case $v in B*) envs="$envs BENCH_SKIP_DONE_WAIT=1";; esac
  env $envs timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu > gpurun_out/bench_r04r_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04r_host_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04r_host_$v.log)"; grep "graph loop host\|device idle\|build done\|count reads" gpurun_out/bench_r04r_host_$v.log | cut -c1-200
done
