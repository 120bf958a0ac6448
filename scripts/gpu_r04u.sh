#!/bin/bash
# Round-4: the host-bound small config (c2: UNet m=16, 4 scenes) with and without the worker-thread prefetch;
# host timing, then interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in A B; do
  extra=""; [ $v = B ] && extra="--prefetch-thread 1"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --preset c2 --steps 30 --warmup 5 --no-cpu $extra > gpurun_out/bench_r04u_c2_host_$v.log 2>&1 || { tail -20 gpurun_out/bench_r04u_c2_host_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_r04u_c2_host_$v.log)"; grep "graph loop host\|device idle\|capture host\|count reads" gpurun_out/bench_r04u_c2_host_$v.log | cut -c1-240
done
TAG=r04u_c2_thread ROUNDS=3 B_LIB=0 BENCH_ARGS="--preset c2 --steps 40 --warmup 5 --no-cpu" B_ARGS="--prefetch-thread 1" bash scripts/gpu_ab.sh || exit 1
