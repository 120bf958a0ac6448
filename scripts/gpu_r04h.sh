#!/bin/bash
# Round-4 A/B: the metadata prefetch on a high-priority stream (bench.py --prefetch-priority 1), C3 and C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r04h_prio ROUNDS=3 ARGS_0="-" ARGS_1="--prefetch-priority 1" BENCH_ARGS="--steps 15 --warmup 5 --no-cpu" bash scripts/gpu_args_ab.sh || exit 1
TAG=r04h_prio_c2 ROUNDS=3 ARGS_0="-" ARGS_1="--prefetch-priority 1" BENCH_ARGS="--preset c2 --steps 20 --warmup 5 --no-cpu" bash scripts/gpu_args_ab.sh || exit 1
BENCH_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 15 --warmup 5 --no-cpu --prefetch-priority 1 > gpurun_out/bench_r04h_c3_host.log 2>&1 || exit 1
grep "graph loop host\|device idle" gpurun_out/bench_r04h_c3_host.log | cut -c1-400
