#!/bin/bash
# Round-4: the library sort's passes, end to end: A = four-launch passes over 4096-pair tiles (the product), B =
# two-launch passes over 16384-pair tiles (lib/libmi3dsparse_exp.so built from the commit before their revert).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r04x_sort ROUNDS=4 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu" bash scripts/gpu_ab.sh || exit 1
