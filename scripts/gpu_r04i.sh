#!/bin/bash
# Round-4 A/B: graph-mode pacing of the metadata prefetch by the step two back (--prefetch-lag 2) vs one back.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r04i_lag ROUNDS=3 ARGS_0="-" ARGS_1="--prefetch-lag 2" BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" bash scripts/gpu_args_ab.sh || exit 1
BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu --prefetch-lag 2 > gpurun_out/bench_r04i_c3_host.log 2>&1 || exit 1
grep "graph loop host\|device idle" gpurun_out/bench_r04i_c3_host.log | cut -c1-400
TAG=r04i_lag_c2 ROUNDS=3 ARGS_0="-" ARGS_1="--prefetch-lag 2" BENCH_ARGS="--preset c2 --steps 30 --warmup 5 --no-cpu" bash scripts/gpu_args_ab.sh || exit 1
